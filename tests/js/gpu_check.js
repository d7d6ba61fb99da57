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
  eng.destroy();
  // luxfhejs-style client
  const cl = new t.LuxFHELocalClient({ params: p });
  await cl.initialize();
  const l = await cl.encrypt_uint8(0b10110011), r = await cl.encrypt_uint8(0b01100110);
  const x = await cl.evaluate({ op: 'xor', left: l, right: r, bitWidth: 8 });
  assert.strictEqual(await cl.decrypt(x, 8), BigInt(0b10110011 ^ 0b01100110));
  cl.close();
  console.log(JSON.stringify({ ok: true }));
})().catch((e) => { console.error(e); process.exit(1); });
