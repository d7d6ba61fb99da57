'use strict';
/**
 * FHE HTTP server on the MI355X engine (SURVEY §8f f2): the endpoint set the reference's JS SDKs
 * call on the external FHE server (default :8448):
 *   GET  /health     -> {status:'ok', threshold, parties, ...}        e2e/test/fhe.test.ts:31-37
 *   GET  /publickey  -> bytes, or {publicKey:number[]} for JSON clients  fhe.test.ts:41-48,
 *                                                                       hardhat-plugin/src/index.ts:84-91
 *   POST /encrypt    {value, bitWidth} -> bytes                          fhe.test.ts:52-78
 *                    {value:string, type:'uint32'|...} -> {ciphertext:number[]}   hardhat-plugin :59-66
 *   POST /evaluate   {op, left:number[], right?:number[]|number, bitWidth} -> bytes   fhe.test.ts:105-175
 *   POST /decrypt    {ciphertext:number[]} -> {value:string}            hardhat-plugin :71-78
 *   POST /verify     bytes -> {verified}                                 fhe.test.ts:179-189
 * Every homomorphic operator runs through js/integer.js on libtfhe_hip.so; /evaluate requests that
 * arrive while the GPU is busy are coalesced and run in lockstep (one PBS launch per circuit level
 * for all of them).  Single-party: this process holds the client key (like the reference's local
 * dev server); /verify checks ciphertext framing only — there is no ZK proof system on this path.
 *
 * --params fhevm_fft serves fhEVM's own representation instead (P-FHEVM radix blocks, js/radix.js:
 * KS -> PBS at N = 2048, every fhEVM operator); the default is gate_fft (boolean gates on the FFT64
 * engine, the one bench.py measures); gate / fhevm run the Goldilocks NTT engine.
 * --devices 0,1,...,7 spreads every batch over those GPUs (one engine shard each, keys broadcast once
 * over RCCL).  Keys and encryptions draw OS entropy; --seed (a public, reproducible key set) is only
 * accepted together with --dev.
 *
 *   node js/server.js [--port 8448] [--host 127.0.0.1] [--devices 0[,1,...]] [--params gate_fft|fhevm_fft|gate|fhevm]
 *                     [--dev --seed 0x7F4E0001]
 */
const http = require('http');

const TYPE_WIDTH = { bool: 1, ebool: 1, uint8: 8, uint16: 16, uint32: 32, uint64: 64, uint128: 128, uint160: 160, uint256: 256, address: 160 };
const MAX_BODY = 256 << 20;

function readBody(req) {
  return new Promise((resolve, reject) => {
    const chunks = [];
    let n = 0;
    req.on('data', (c) => {
      n += c.length;
      if (n > MAX_BODY) { reject(Object.assign(new Error('request body too large'), { status: 413 })); req.destroy(); return; }
      chunks.push(c);
    });
    req.on('end', () => resolve(Buffer.concat(chunks)));
    req.on('error', reject);
  });
}

function sendJson(res, status, obj) {
  const body = Buffer.from(JSON.stringify(obj));
  res.writeHead(status, { 'Content-Type': 'application/json', 'Content-Length': body.length });
  res.end(body);
}

function sendBytes(res, bytes) {
  const body = Buffer.from(bytes.buffer, bytes.byteOffset, bytes.byteLength);
  res.writeHead(200, { 'Content-Type': 'application/octet-stream', 'Content-Length': body.length });
  res.end(body);
}

const wantsJsonOnly = (req) => /^application\/json/i.test(req.headers.accept || '');

function toBytes(x, field) {
  if (Array.isArray(x)) return Uint8Array.from(x);
  if (typeof x === 'string') return Uint8Array.from(Buffer.from(x, 'base64'));
  throw Object.assign(new Error(`${field}: expected a byte array`), { status: 400 });
}

/** client: an initialized LuxFHELocalClient (js/index.js) or any object with the same methods */
function createServer(client, info = {}) {
  return http.createServer(async (req, res) => {
    try {
      const url = (req.url || '/').split('?')[0];
      if (req.method === 'GET' && url === '/health') {
        return sendJson(res, 200, { status: 'ok', threshold: 1, parties: 1, backend: 'libtfhe_hip (gfx950)', ...info });
      }
      if (req.method === 'GET' && url === '/publickey') {
        const pk = await client.getPublicKey();
        return wantsJsonOnly(req) ? sendJson(res, 200, { publicKey: Array.from(pk) }) : sendBytes(res, pk);
      }
      if (req.method !== 'POST') return sendJson(res, 404, { error: `no route ${req.method} ${url}` });
      const raw = await readBody(req);
      if (url === '/verify') {
        // framing check: a tfhe_amd ciphertext must parse; other (proof) bytes: non-empty
        let verified = raw.length > 0;
        if (raw.length >= 4 && raw.readUInt32LE(0) === 0x31414654) {
          try { require('./index.js').parseCiphertext(new Uint8Array(raw)); } catch (e) { verified = false; }
        }
        return sendJson(res, 200, { verified });
      }
      let body;
      try { body = JSON.parse(raw.toString('utf8') || '{}'); } catch (e) { return sendJson(res, 400, { error: 'invalid JSON body' }); }
      if (url === '/encrypt') {
        if (body.value === undefined) return sendJson(res, 400, { error: 'value required' });
        if (body.type !== undefined) {
          const w = TYPE_WIDTH[String(body.type).toLowerCase()];
          if (!w) return sendJson(res, 400, { error: `unsupported type ${body.type}` });
          return sendJson(res, 200, { ciphertext: Array.from(client.encryptValue(body.value, w)) });
        }
        const w = Number(body.bitWidth || 32);
        if (!(w >= 1 && w <= 256)) return sendJson(res, 400, { error: `unsupported bitWidth ${body.bitWidth}` });
        return sendBytes(res, client.encryptValue(body.value, w));
      }
      if (url === '/evaluate') {
        if (!body.op || body.left === undefined) return sendJson(res, 400, { error: 'op and left required' });
        const right = body.right === undefined || body.right === null ? null
          : (typeof body.right === 'number' || (typeof body.right === 'string' && /^\d+$/.test(body.right)) ? BigInt(body.right) : toBytes(body.right, 'right'));
        const out = await client.evaluate({ op: body.op, left: toBytes(body.left, 'left'), right, bitWidth: body.bitWidth });
        return sendBytes(res, out);
      }
      if (url === '/decrypt') {
        if (body.ciphertext === undefined) return sendJson(res, 400, { error: 'ciphertext required' });
        const v = await client.decrypt(toBytes(body.ciphertext, 'ciphertext'));
        return sendJson(res, 200, { value: v.toString() });
      }
      return sendJson(res, 404, { error: `no route POST ${url}` });
    } catch (e) {
      return sendJson(res, e.status || 400, { error: e.message });
    }
  });
}

module.exports = { createServer };

if (require.main === module) {
  const args = process.argv.slice(2);
  const opt = (name, dflt) => { const i = args.indexOf(`--${name}`); return i >= 0 ? args[i + 1] : dflt; };
  const { LuxFHELocalClient } = require('./index.js');
  const params = opt('params', 'gate_fft');
  const devices = String(opt('devices', opt('device', '0'))).split(',').map(Number);
  const dev = args.includes('--dev');
  const seed = opt('seed', undefined);
  if (seed !== undefined && !dev) {
    console.error('--seed makes every key and ciphertext reproducible by anyone who knows it: add --dev to accept that');
    process.exit(2);
  }
  let client;
  try {
    client = new LuxFHELocalClient({ devices, seed: seed === undefined ? undefined : BigInt(seed), dev, params });
  } catch (e) { console.error(e.message); process.exit(2); }
  client.initialize().then(() => {
    const port = Number(opt('port', 8448)), host = opt('host', '127.0.0.1');
    createServer(client, { device: devices[0], devices, params }).listen(port, host, () => {
      console.log(`tfhe_amd FHE server (${params}, devices ${devices.join(',')}) on http://${host}:${port}`);
    });
  }).catch((e) => { console.error(e); process.exit(1); });
}
