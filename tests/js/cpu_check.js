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
console.log(JSON.stringify(out));
