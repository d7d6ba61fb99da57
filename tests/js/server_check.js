'use strict';
// HTTP server check (js/server.js) with the request shapes of the reference's e2e test
// (e2e/test/fhe.test.ts) and hardhat plugin.  argv[2] === 'gpu': the real MI355X engine;
// otherwise a key-holding test double stands in for the gate bootstrap (CPU: phase -> sign ->
// trivial ciphertext), so the host logic (routes, framing, coalescing, circuits) runs without a GPU.
// argv[2] === 'fhevm' / 'fhevm-gpu': the same requests on P-FHEVM radix blocks (js/radix.js); the
// CPU double decrypts each block and applies the bootstrap's table.
const path = require('path');
const http = require('http');
const assert = require('assert');
const tfhe = require(path.join(__dirname, '..', '..', 'js', 'index.js'));
const { createServer } = require(path.join(__dirname, '..', '..', 'js', 'server.js'));

const mode = process.argv[2] || 'cpu';
const useGpu = mode === 'gpu' || mode === 'fhevm-gpu';
const fhevm = mode.startsWith('fhevm');
const HALF = 1n << 63n;

function request(port, method, url, body, headers = {}) {
  return new Promise((resolve, reject) => {
    const data = body === undefined ? null : (Buffer.isBuffer(body) || body instanceof Uint8Array ? Buffer.from(body) : Buffer.from(JSON.stringify(body)));
    const req = http.request({ host: '127.0.0.1', port, method, path: url, headers: { 'Content-Type': Buffer.isBuffer(body) ? 'application/octet-stream' : 'application/json', ...headers } }, (res) => {
      const chunks = [];
      res.on('data', (c) => chunks.push(c));
      res.on('end', () => resolve({ status: res.statusCode, type: res.headers['content-type'], body: Buffer.concat(chunks) }));
    });
    req.on('error', reject);
    if (data) req.write(data);
    req.end();
  });
}

(async () => {
  let client;
  const dbl = {
    params: tfhe.paramsPreset(tfhe.PRESET_GATE),
    gateLut() { return null; },
    calls: 0,
    async pbs(cts) {
      this.calls++;
      const d = this.params.n + 1;
      const ph = client.clientKey.phase(cts);
      const out = new BigUint64Array(cts.length);
      for (let i = 0; i < ph.length; i++) out[(i + 1) * d - 1] = (ph[i] !== 0n && ph[i] < HALF) ? tfhe.MU : (1n << 64n) - tfhe.MU;
      return out;
    },
  };
  const rdbl = {
    params: tfhe.paramsPreset(tfhe.PRESET_FHEVM),
    lutFromTable(t) { return BigUint64Array.from(t, BigInt); },
    calls: 0,
    async pbs(cts, luts, idx) {
      this.calls++;
      const d = this.params.k * this.params.N + 1;
      const v = client.clientKey.decrypt(cts, 16);
      const out = new BigUint64Array(cts.length);
      for (let i = 0; i < v.length; i++) out[(i + 1) * d - 1] = luts[idx[i] * this.params.N + v[i]] * tfhe.radix.DELTA;
      return out;
    },
  };
  // GPU: the server defaults (FFT64 engines), spread over two shards of device 0 (the --devices split)
  const cfg = fhevm ? { params: useGpu ? 'fhevm_fft' : 'fhevm' } : {};
  if (useGpu) cfg.devices = [0, 0];
  if (!useGpu) cfg.engine = fhevm ? rdbl : dbl;
  client = new tfhe.LuxFHELocalClient(cfg);
  const ctBytes = (w) => 16 + 8 * (fhevm ? (w / 2) * 2049 : w * 631);
  await client.initialize();
  const server = createServer(client).listen(0, '127.0.0.1');
  await new Promise((r) => server.on('listening', r));
  const port = server.address().port;
  try {
    let r = await request(port, 'GET', '/health');
    assert.strictEqual(JSON.parse(r.body).status, 'ok');
    r = await request(port, 'GET', '/publickey', undefined, { Accept: '*/*' });
    assert.ok(r.body.length > 0 && /octet-stream/.test(r.type));
    r = await request(port, 'GET', '/publickey', undefined, { Accept: 'application/json, text/plain, */*' });
    assert.ok(JSON.parse(r.body).publicKey.length > 0);
    for (const w of [8, 16, 32, 64]) {
      r = await request(port, 'POST', '/encrypt', { value: 123, bitWidth: w });
      assert.strictEqual(r.status, 200);
      assert.strictEqual(r.body.length, ctBytes(w));
    }
    const encA = (await request(port, 'POST', '/encrypt', { value: 42, bitWidth: 32 })).body;
    const encB = (await request(port, 'POST', '/encrypt', { value: 17, bitWidth: 32 })).body;
    const dec = async (bytes) => BigInt(JSON.parse((await request(port, 'POST', '/decrypt', { ciphertext: Array.from(bytes) })).body).value);
    assert.strictEqual(await dec(encA), 42n);
    // the four /evaluate calls of fhe.test.ts, submitted concurrently (coalesced into shared launches)
    const ev = (op, left, right) => request(port, 'POST', '/evaluate', { op, left: Array.from(left), right: Array.from(right), bitWidth: 32 });
    const [add, sub, lt, eq] = await Promise.all([ev('add', encA, encB), ev('sub', encA, encB), ev('lt', encA, encB), ev('eq', encA, encA)]);
    for (const x of [add, sub, lt, eq]) assert.strictEqual(x.status, 200, x.body.toString());
    assert.strictEqual(await dec(add.body), 59n);
    assert.strictEqual(await dec(sub.body), 25n);
    assert.strictEqual(await dec(lt.body), 0n);
    assert.strictEqual(await dec(eq.body), 1n);
    // scalar right operand, mul, min
    r = await request(port, 'POST', '/evaluate', { op: 'mul', left: Array.from(encB), right: 3, bitWidth: 32 });
    assert.strictEqual(await dec(r.body), 51n);
    // hardhat plugin shapes
    r = await request(port, 'POST', '/encrypt', { value: '200', type: 'uint8' });
    const hh = JSON.parse(r.body).ciphertext;
    assert.strictEqual(JSON.parse((await request(port, 'POST', '/decrypt', { ciphertext: hh })).body).value, '200');
    // verify + errors
    r = await request(port, 'POST', '/verify', Buffer.from([1, 2, 3]));
    assert.strictEqual(JSON.parse(r.body).verified, true);
    // shifts / rotations (plaintext and encrypted amounts), neg, bitwise, max
    const enc5 = (await request(port, 'POST', '/encrypt', { value: 5, bitWidth: 8 })).body;
    const [shl, rotr, shlE, neg, xor, mx] = await Promise.all([
      request(port, 'POST', '/evaluate', { op: 'shl', left: Array.from(encA), right: 3, bitWidth: 32 }),
      request(port, 'POST', '/evaluate', { op: 'rotr', left: Array.from(encB), right: 4, bitWidth: 32 }),
      ev('shl', encB, enc5), request(port, 'POST', '/evaluate', { op: 'neg', left: Array.from(encB), bitWidth: 32 }),
      ev('xor', encA, encB), ev('max', encA, encB)]);
    assert.strictEqual(await dec(shl.body), 42n << 3n);
    assert.strictEqual(await dec(rotr.body), ((17n >> 4n) | (17n << 28n)) & 0xFFFFFFFFn);
    assert.strictEqual(await dec(shlE.body), 17n << 5n);
    assert.strictEqual(await dec(neg.body), (1n << 32n) - 17n);
    assert.strictEqual(await dec(xor.body), 42n ^ 17n);
    assert.strictEqual(await dec(mx.body), 42n);
    // ebool
    const t = (await request(port, 'POST', '/encrypt', { value: 1, bitWidth: 1 })).body;
    const f = (await request(port, 'POST', '/encrypt', { value: 0, bitWidth: 1 })).body;
    const [band, bor, bnot] = await Promise.all([ev('and', t, f), ev('or', t, f),
      request(port, 'POST', '/evaluate', { op: 'not', left: Array.from(f), bitWidth: 1 })]);
    assert.strictEqual(await dec(band.body), 0n);
    assert.strictEqual(await dec(bor.body), 1n);
    assert.strictEqual(await dec(bnot.body), 1n);
    r = await request(port, 'POST', '/evaluate', { op: 'pow', left: Array.from(encA), right: Array.from(encB), bitWidth: 32 });
    assert.strictEqual(r.status, 400);
    r = await request(port, 'POST', '/decrypt', { ciphertext: [1, 2, 3] });
    assert.strictEqual(r.status, 400);
    console.log(`OK server (${useGpu ? 'gpu' : 'cpu double'}${fhevm ? ', fhevm radix' : ''}), evaluate launches ${client.launches}`);
  } finally {
    server.close();
    client.close();
  }
})().catch((e) => { console.error(e); process.exit(1); });
