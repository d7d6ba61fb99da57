'use strict';
// HTTP server check (js/server.js) with the request shapes of the reference's e2e test
// (e2e/test/fhe.test.ts) and hardhat plugin.  argv[2] === 'gpu': the real MI355X engine;
// otherwise a key-holding test double stands in for the gate bootstrap (CPU: phase -> sign ->
// trivial ciphertext), so the host logic (routes, framing, coalescing, circuits) runs without a GPU.
const path = require('path');
const http = require('http');
const assert = require('assert');
const tfhe = require(path.join(__dirname, '..', '..', 'js', 'index.js'));
const { createServer } = require(path.join(__dirname, '..', '..', 'js', 'server.js'));

const useGpu = process.argv[2] === 'gpu';
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
  client = new tfhe.LuxFHELocalClient(useGpu ? {} : { engine: dbl });
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
      assert.strictEqual(r.body.length, 16 + 8 * w * 631);
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
    r = await request(port, 'POST', '/evaluate', { op: 'pow', left: Array.from(encA), right: Array.from(encB), bitWidth: 32 });
    assert.strictEqual(r.status, 400);
    r = await request(port, 'POST', '/decrypt', { ciphertext: [1, 2, 3] });
    assert.strictEqual(r.status, 400);
    console.log(`OK server (${useGpu ? 'gpu' : 'cpu double'}), evaluate launches ${client.launches}`);
  } finally {
    server.close();
    client.close();
  }
})().catch((e) => { console.error(e); process.exit(1); });
