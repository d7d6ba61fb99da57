'use strict';
// CPU check of js/integer.js: every fhEVM KAT (tests/golden/fhevm_kats.json) through the JS
// operator layer with a cleartext test double for the gate bootstrap (trivial ciphertexts only:
// the phase is the body; asserts >= 1/16 torus margin on every gate), all KATs in lockstep.
const path = require('path');
const assert = require('assert');
const I = require(path.join(__dirname, '..', '..', 'js', 'integer.js'));
const kats = require(path.join(__dirname, '..', 'golden', 'fhevm_kats.json'));

const HALF = 1n << 63n;
let minMargin = 1n << 62n;
// trivial ciphertexts: the mask width does not matter, so the double runs at n = 0 (body only) to keep
// the euint128 multiplier levels (~10^6 gates) in memory
const D = 1;
const engine = {
  params: { n: D - 1 },
  gateLut() { return null; },
  async pbs(cts) {
    const d = D;
    const out = new BigUint64Array(cts.length);
    for (let i = 0; i < cts.length; i += d) {
      for (let j = 0; j < d - 1; j++) assert.strictEqual(cts[i + j], 0n, 'trivial ciphertexts only');
      const b = cts[i + d - 1];
      const d0 = b < HALF ? b : (1n << 64n) - b;
      const d1 = b < HALF ? HALF - b : b - HALF;
      const m = d0 < d1 ? d0 : d1;
      if (m < minMargin) minMargin = m;
      out[i + d - 1] = (b !== 0n && b < HALF) ? I.MU : (1n << 64n) - I.MU;
    }
    return out;
  },
};
const clearKey = { decryptBool(col) { const r = []; for (let i = D - 1; i < col.length; i += D) r.push(col[i] !== 0n && col[i] < HALF); return r; } };
const width = (t) => (t === 'ebool' ? 1 : Number(t.replace('euint', '').replace('uint', '')));

(async () => {
  const c = new I.Circuit(engine);
  const gens = kats.map((k) => {
    const args = k.types.map((t, i) => (t.startsWith('e') ? I.FheUintVec.trivial(c, [BigInt(k.args[i])], width(t)) : BigInt(k.args[i])));
    return I.fhevmOp(c, k.op, ...args);
  });
  const res = await c.runMany(gens);
  let bad = 0;
  kats.forEach((k, i) => {
    let got;
    if (k.result_type === 'ebool') got = clearKey.decryptBool(res[i])[0] ? 1n : 0n;
    else got = res[i].decrypt(clearKey)[0];
    const want = k.result_type === 'ebool' ? (BigInt(k.expect) ? 1n : 0n) : BigInt(k.expect);
    if (got !== want) { bad++; if (bad < 5) console.error('KAT mismatch', k.source, k.op, k.types, k.args, want, got); }
  });
  assert.strictEqual(bad, 0, `${bad} KATs failed`);
  assert.ok(minMargin >= (1n << 60n), `margin ${minMargin}`);
  assert.ok(c.launches < 400, `launches ${c.launches}`);
  // ripple path on a batch, and value-major round trip
  const c2 = new I.Circuit(engine, 4);
  const A = I.FheUintVec.trivial(c2, [250n, 7n, 0n, 65535n], 16), Bv = I.FheUintVec.trivial(c2, [9n, 7n, 1n, 1n], 16);
  const [s, lt] = await c2.runMany([I.fhevmOp(c2, 'add', A, Bv), I.fhevmOp(c2, 'lt', A, Bv)]);
  assert.deepStrictEqual(s.decrypt(clearKey), [259n, 14n, 1n, 0n]);
  assert.deepStrictEqual(clearKey.decryptBool(lt), [false, false, true, false]);
  const rt = I.FheUintVec.fromValueMajor(c2, A.toValueMajor(), 4, 16);
  assert.deepStrictEqual(rt.decrypt(clearKey), [250n, 7n, 0n, 65535n]);
  console.log(`OK ${kats.length} KATs, ${c.launches} launches, ${c.pbsCount} PBS`);
})().catch((e) => { console.error(e); process.exit(1); });
