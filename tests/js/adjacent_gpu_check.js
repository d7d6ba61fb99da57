// The adjacent fhEVM kernels through the N-API boundary on the GPU (tests/test_js.py::test_js_adjacent_gpu):
// ciphertext compression (Packer: packing keyswitch + modulus-switched bit packing) and noise squashing
// (Squasher: keyswitch + MS noise reduction on the P-FHEVM engine, then the 128-bit bootstrap).  Inputs come from
// the pytest side (raw little-endian u64 files in DIR); outputs are written back for a byte-for-byte comparison with
// the Python / ctypes path.  Prints one JSON line.
const fs = require('fs');
const path = require('path');
const assert = require('assert');
const t = require('../../js');

const rd = (f) => { const b = fs.readFileSync(f); return new BigUint64Array(b.buffer, b.byteOffset, b.length / 8); };
const wr = (f, a) => fs.writeFileSync(f, Buffer.from(a.buffer, a.byteOffset, a.byteLength));

(async () => {
  const dir = process.argv[2];
  const seed = BigInt(process.argv[3]);
  const res = {};
  // ---- compression
  const inKey = rd(path.join(dir, 'in_key.bin'));
  const lwes = rd(path.join(dir, 'lwes.bin'));
  const { outKey, pksk } = t.Packer.keygen(inKey, seed);
  const packer = new t.Packer(0).loadKey(pksk);
  const groups = await packer.packCompress(lwes);
  const glwes = new BigUint64Array(groups.length * 4096);
  groups.forEach((g, i) => glwes.set(g.glwe, i * 4096));
  wr(path.join(dir, 'js_glwes.bin'), glwes);
  wr(path.join(dir, 'js_packed.bin'), BigUint64Array.from(groups.flatMap((g) => Array.from(g.packed))));
  wr(path.join(dir, 'js_out_key.bin'), outKey);
  // decompress the last (ragged) GLWE and check it against the packed one within the storage precision
  const last = groups[groups.length - 1];
  const back = t.Packer.extract(last.packed, last.bodies);
  const ph = t.Packer.glwePhase(outKey, back), ph0 = t.Packer.glwePhase(outKey, last.glwe);
  let maxd = 0n;
  for (let j = 0; j < last.bodies; j++) {
    let d = BigInt.asIntN(64, ph[j] - ph0[j]);
    if (d < 0n) d = -d;
    if (d > maxd) maxd = d;
  }
  res.groups = groups.length;
  res.extract_max_err_log2 = maxd === 0n ? 0 : maxd.toString(2).length;
  packer.destroy();
  // ---- noise squashing on P-FHEVM (FFT64 engine)
  const p = t.paramsPreset(t.PRESET_FHEVM_FFT);
  const [ck, sk] = t.genKeys(p, seed);
  const eng = new t.Engine(p, 0).loadKeys(sk);
  const { glweKey, bsk } = t.Squasher.keygen(ck.lweKey, seed);
  const sq = new t.Squasher(0).loadKey(bsk);
  const msgs = Array.from({ length: 64 }, (_, i) => (i * 7 + 3) % 16);
  const cts = ck.encrypt(msgs, 16, seed + 1n);
  // a modulus the squashing LUT cannot take throws synchronously, before any GPU work is queued
  for (const bad of [0, 3, 4096]) assert.throws(() => sq.squash(eng, cts, bad), /msgModulus/);
  res.squash_bad_modulus_sync_throw = true;
  const out = await sq.squash(eng, cts, 16);
  wr(path.join(dir, 'js_squash.bin'), out);
  assert.deepStrictEqual(t.Squasher.decrypt(glweKey, out, 16), msgs);
  res.squash_decrypt_ok = true;
  // a squash and a PBS in flight together on the same engine
  const [o2, pb] = await Promise.all([sq.squash(eng, cts.subarray(0, 2049 * 4), 16),
    eng.pbs(cts.subarray(0, 2049 * 4), eng.lutFromTable(Array.from({ length: 16 }, (_, m) => m)))]);
  assert.deepStrictEqual(t.Squasher.decrypt(glweKey, o2, 16), msgs.slice(0, 4));
  assert.deepStrictEqual(ck.decrypt(pb, 16), msgs.slice(0, 4));
  sq.destroy();
  eng.destroy();
  res.ok = true;
  console.log(JSON.stringify(res));
})().catch((e) => { console.error(e); process.exit(1); });
