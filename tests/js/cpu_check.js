// CPU-side checks of the N-API addon (no GPU): exports, key material, encrypt/phase, errors.
// Prints one JSON line consumed by tests/test_js.py.
const assert = require('assert');
const crypto = require('crypto');
const t = require('../../js');

const out = {};
out.exports = Object.keys(t.native).sort();
const p = t.paramsPreset(t.PRESET_GATE);
assert.strictEqual(p.n, 630); assert.strictEqual(p.N, 1024);
const [ck, sk] = t.genKeys(p, 0x7F4E0001n);
const h = (a) => crypto.createHash('sha256').update(Buffer.from(a.buffer, a.byteOffset, a.byteLength)).digest('hex');
out.lwe_key_sha = h(ck.lweKey);
out.bsk_sha = h(sk.bsk);
out.ksk_sha = h(sk.ksk);
const cts = ck.encryptBool([true, false, true], 0xC0FFEE02n, 5n);
out.ct_sha = h(cts);
assert.deepStrictEqual(ck.decryptBool(cts), [true, false, true]);
const m = ck.encrypt([0, 1, 2, 3], 4, 9n);
assert.deepStrictEqual(ck.decrypt(m, 4), [0, 1, 2, 3]);
try { t.native.lutFromTable(1024, 3, new BigUint64Array(3), 1n); out.err = 'none'; } catch (e) { out.err = e.code; }
try { new t.Engine(p, 0); out.engine = 'created'; } catch (e) { out.engine = e.code; }
// production defaults draw OS entropy: fresh keys and fresh encryption randomness every call
const [ck1] = t.genKeys(p), [ck2] = t.genKeys(p);
out.entropy_keys_differ = h(ck1.lweKey) !== h(ck2.lweKey);
const e1 = ck1.encryptBool([true]), e2 = ck1.encryptBool([true]);
out.entropy_cts_differ = h(e1) !== h(e2) && ck1.decryptBool(e1)[0] && ck1.decryptBool(e2)[0];
try { new t.LuxFHELocalClient({ seed: 1n }); out.seed_refused = false; } catch (e) { out.seed_refused = /dev: true/.test(e.message); }
out.seed_dev_ok = new t.LuxFHELocalClient({ seed: 1n, dev: true }).seed === 1n;
out.default_params = new t.LuxFHELocalClient().params.transform;
// unseal(contractAddress, sealedData): bigint, synchronous like luxfhejs (index.ts:146); the client key is host-side
{
  const cl = new t.LuxFHELocalClient({ seed: 7n, dev: true, params: p });
  [cl.clientKey] = t.genKeys(cl.params, 7n);
  const sealed = cl.encryptValue(0xA5, 8);
  const u = cl.unseal('0x00000000000000000000000000000000000000aa', sealed);
  out.unseal_sync = typeof u === 'bigint' && u === 0xA5n
    && cl.unseal('0xaa', '0x' + Buffer.from(sealed).toString('hex')) === 0xA5n;
}
console.log(JSON.stringify(out));
