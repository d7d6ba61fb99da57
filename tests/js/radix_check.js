'use strict';
// CPU check of js/radix.js: every fhEVM KAT (tests/golden/fhevm_kats.json) with a cleartext
// double of the multi-LUT PBS on trivial blocks (asserts no block ever reaches the padding bit),
// all KATs in lockstep; then a random batch per operator (div/rem over several divisors).
// Prints "OK <kats> <launches> <pbs>" — tests/test_js.py compares the counts with tfhe_amd/radix.py.
const path = require('path');
const assert = require('assert');
const R = require(path.join(__dirname, '..', '..', 'js', 'radix.js'));
const kats = require(path.join(__dirname, '..', 'golden', 'fhevm_kats.json')).filter((k) => R.RADIX_OPS.includes(k.op));

// trivial blocks: the mask width does not matter; N = 16 (one table entry per coefficient) keeps the
// euint128 levels in memory
const N = 16, DIM = N + 1;
let maxSeen = 0;
const engine = {
  params: { k: 1, N, n: 918, order: 1 },
  lutFromTable(t) { return BigUint64Array.from(t, BigInt); }, // the double keeps the table itself
  async pbs(cts, luts, idx) {
    const out = new BigUint64Array(cts.length);
    for (let b = 0; b < cts.length / DIM; b++) {
      for (let j = 0; j < DIM - 1; j++) assert.strictEqual(cts[b * DIM + j], 0n, 'trivial blocks only');
      const body = cts[(b + 1) * DIM - 1];
      assert.strictEqual(body % R.DELTA, 0n);
      const v = Number(body / R.DELTA);
      assert.ok(v < R.SPACE, `block value ${v} crossed the padding bit`);
      maxSeen = Math.max(maxSeen, v);
      out[(b + 1) * DIM - 1] = luts[idx[b] * N + v] * R.DELTA;
    }
    return out;
  },
};
const clearKey = { decrypt(col, mm) { const r = []; for (let i = DIM - 1; i < col.length; i += DIM) r.push(Number((col[i] / R.DELTA) % BigInt(mm))); return r; } };
const width = (t) => (t === 'ebool' ? 1 : Number(t.replace('euint', '').replace('uint', '')));

(async () => {
  const c = new R.RadixCircuit(engine);
  const gens = kats.map((k) => {
    const args = k.types.map((t, i) => (t.startsWith('e') ? R.RadixVec.trivial(c, [BigInt(k.args[i])], width(t)) : BigInt(k.args[i])));
    return R.fhevmOp(c, k.op, ...args);
  });
  const res = await c.runMany(gens);
  let bad = 0;
  kats.forEach((k, i) => {
    let got;
    if (k.result_type === 'ebool') got = BigInt(clearKey.decrypt(res[i], 16)[0]);
    else { got = BigInt(R.decryptRadix(clearKey, res[i])[0]); assert.strictEqual(res[i].width, width(k.result_type)); }
    const want = k.result_type === 'ebool' ? (BigInt(k.expect) ? 1n : 0n) : BigInt(k.expect);
    if (got !== want) { bad++; if (bad < 5) console.error('KAT mismatch', k.source, k.op, k.types, k.args, want, got); }
  });
  assert.strictEqual(bad, 0, `${bad} KATs failed`);
  assert.ok(maxSeen <= 15);
  const katLaunches = c.launches, katPbs = c.pbsCount;

  // random batch, every operator, w = 16
  const w = 16, B = 24, m = (1n << 16n) - 1n;
  let s = 12345n;
  const rnd = () => { s = (s * 6364136223846793005n + 1442695040888963407n) & ((1n << 64n) - 1n); return (s >> 20n) & m; };
  const a = Array.from({ length: B }, rnd), b = Array.from({ length: B }, rnd);
  b[0] = a[0];
  const c2 = new R.RadixCircuit(engine);
  const A = R.RadixVec.trivial(c2, a, w), Bv = R.RadixVec.trivial(c2, b, w);
  const rot = (x, k, l) => (l ? ((x << k) | (x >> (16n - k))) & m : ((x >> k) | (x << (16n - k))) & m);
  const want = {
    add: (x, y) => (x + y) & m, sub: (x, y) => (x - y) & m, mul: (x, y) => (x * y) & m, and: (x, y) => x & y,
    or: (x, y) => x | y, xor: (x, y) => x ^ y, min: (x, y) => (x < y ? x : y), max: (x, y) => (x > y ? x : y),
    eq: (x, y) => BigInt(x === y), ne: (x, y) => BigInt(x !== y), lt: (x, y) => BigInt(x < y), le: (x, y) => BigInt(x <= y),
    gt: (x, y) => BigInt(x > y), ge: (x, y) => BigInt(x >= y),
    shl: (x, y) => (x << (y % 16n)) & m, shr: (x, y) => x >> (y % 16n), rotl: (x, y) => rot(x, y % 16n, true), rotr: (x, y) => rot(x, y % 16n, false),
  };
  const ops = Object.keys(want);
  const out = await c2.runMany(ops.map((op) => R.fhevmOp(c2, op, A, Bv)));
  ops.forEach((op, i) => {
    const r = out[i];
    const got = r instanceof R.RadixVec ? R.decryptRadix(clearKey, r) : clearKey.decrypt(r, 16).map(BigInt);
    a.forEach((x, j) => assert.strictEqual(got[j], want[op](x, b[j]), `${op} ${x} ${b[j]}`));
  });
  const [neg, not, shl5] = await c2.runMany([R.fhevmOp(c2, 'neg', A), R.fhevmOp(c2, 'not', A), R.fhevmOp(c2, 'shl', A, 5n)]);
  assert.deepStrictEqual(R.decryptRadix(clearKey, neg), a.map((x) => (0n - x) & m));
  assert.deepStrictEqual(R.decryptRadix(clearKey, not), a.map((x) => x ^ m));
  assert.deepStrictEqual(R.decryptRadix(clearKey, shl5), a.map((x) => (x << 5n) & m));
  for (const d of [0n, 1n, 4n, 7n, 8n, 1000n, 65535n]) {
    const [q, r] = await c2.runMany([R.fhevmOp(c2, 'div', A, d), R.fhevmOp(c2, 'rem', A, d)]);
    assert.deepStrictEqual(R.decryptRadix(clearKey, q), a.map((x) => (d === 0n ? m : x / d)), `div ${d}`);
    assert.deepStrictEqual(R.decryptRadix(clearKey, r), a.map((x) => (d === 0n ? x : x % d)), `rem ${d}`);
  }
  const rt = R.RadixVec.fromValueMajor(c2, A.toValueMajor(), B, 8);
  assert.deepStrictEqual(R.decryptRadix(clearKey, rt), a);
  console.log(`OK ${kats.length} ${katLaunches} ${katPbs}`);
})().catch((e) => { console.error(e); process.exit(1); });
