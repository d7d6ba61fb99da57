// GPU checks through the N-API addon: NAND truth table, FheBool gates, FheUint8 xor, LUT PBS,
// LuxFHELocalClient evaluate round trip.  Prints one JSON line (tests/test_js.py).
const assert = require('assert');
const t = require('../../js');

(async () => {
  const p = t.paramsPreset(Number(process.argv[2] || t.PRESET_GATE));  // 0: NTT engine, 2: FFT64 engine
  const [ck, sk] = t.genKeys(p, 0x7F4E0001n);
  const eng = new t.Engine(p, 0).loadKeys(sk);
  const a = [false, false, true, true], b = [false, true, false, true];
  const A = t.FheBool.encrypt(a, ck, eng, 1n), B = t.FheBool.encrypt(b, ck, eng, 2n);
  assert.deepStrictEqual((await A.nand(B)).decrypt(ck), a.map((x, i) => !(x && b[i])));
  assert.deepStrictEqual((await A.and(B)).decrypt(ck), a.map((x, i) => x && b[i]));
  assert.deepStrictEqual((await A.or(B)).decrypt(ck), a.map((x, i) => x || b[i]));
  assert.deepStrictEqual((await A.xor(B)).decrypt(ck), a.map((x, i) => x !== b[i]));
  assert.deepStrictEqual(A.not().decrypt(ck), a.map((x) => !x));
  const X = t.FheUint8.encrypt([71, 66], ck, eng, 3n), Y = t.FheUint8.encrypt([66, 200], ck, eng, 4n);
  assert.deepStrictEqual((await X.xor(Y)).decrypt(ck), [71n ^ 66n, 66n ^ 200n]);
  // biometrics main.rs:65-77: popcount LUT over all 8 messages
  const f = (m) => m.toString(2).split('1').length - 1;
  const msgs = [0, 1, 2, 3, 4, 5, 6, 7];
  const ct = ck.encrypt(msgs, 8, 7n);
  const acc = eng.generateAccumulator(f, 8);
  const res = await eng.keyswitchProgrammableBootstrap(ct, acc);
  assert.deepStrictEqual(ck.decrypt(res, 8), msgs.map((m) => f(m) % 8));
  // several PBS in flight from the event loop
  const many = await Promise.all([0, 1, 2].map(() => eng.pbs(ct, acc)));
  for (const r of many) assert.deepStrictEqual(ck.decrypt(r, 8), msgs.map((m) => f(m) % 8));
  // stage-level calls: blind rotation alone, keyswitch alone (P-GATE: PBS = KS(SE(BR)))
  const br = await eng.blindRotate(ct, acc);
  assert.strictEqual(br.length, msgs.length * 2 * p.N);
  const big = new BigUint64Array(msgs.length * (p.N + 1));  // sample extract on the host: a_j = -A[N-j]
  for (let q = 0; q < msgs.length; q++) {
    const A = br.subarray(q * 2 * p.N, q * 2 * p.N + p.N), Bp = br.subarray(q * 2 * p.N + p.N, (q + 1) * 2 * p.N);
    const o = big.subarray(q * (p.N + 1), (q + 1) * (p.N + 1));
    o[0] = A[0];
    for (let j = 1; j < p.N; j++) o[j] = BigInt.asUintN(64, -A[p.N - j]);
    o[p.N] = Bp[0];
  }
  if (p.transform === 1) {  // FFT64 accumulators are native-torus values: extract + keyswitch == pbs
    const ks = await eng.keyswitch(big);
    assert.deepStrictEqual(Array.from(ks), Array.from(res));
  }
  // destroy while a job is in flight: the job still completes (the ctx outlives it), then it is gone
  const inflight = eng.pbs(ct, acc);
  eng.destroy();
  assert.deepStrictEqual(ck.decrypt(await inflight, 8), msgs.map((m) => f(m) % 8));
  // two shards of device 0: the batch splits across them, keys reach shard 1 by device copy
  const eng2 = new t.Engine(p, [0, 0]).loadKeys(sk);
  const info = eng2.info();
  assert.deepStrictEqual(info.devices, [0, 0]);
  assert.strictEqual(info.keyBroadcast, 'copy');
  const r2 = await eng2.pbs(ct, acc);
  assert.deepStrictEqual(Array.from(r2), Array.from(res));
  eng2.destroy();
  // luxfhejs-style client
  const cl = new t.LuxFHELocalClient({ params: p, devices: [0, 0] });
  await cl.initialize();
  const l = await cl.encrypt_uint8(0b10110011), r = await cl.encrypt_uint8(0b01100110);
  const x = await cl.evaluate({ op: 'xor', left: l, right: r, bitWidth: 8 });
  assert.strictEqual(await cl.decrypt(x, 8), BigInt(0b10110011 ^ 0b01100110));
  // unseal is synchronous like the reference's (luxfhejs index.ts:146): a bigint, not a Promise; bytes or hex
  const u = cl.unseal('0x00000000000000000000000000000000000000aa', x);
  assert.strictEqual(typeof u, 'bigint');
  assert.strictEqual(u, BigInt(0b10110011 ^ 0b01100110));
  assert.strictEqual(cl.unseal('0xaa', '0x' + Buffer.from(x).toString('hex')), u);
  cl.close();
  console.log(JSON.stringify({ ok: true }));
})().catch((e) => { console.error(e); process.exit(1); });
