'use strict';
/**
 * @luxfhe-amd/tfhe — JS host side of the MI355X PBS engine.
 *
 * Drop-in for the TFHE core the reference's JS reaches (packages/wasm = tfhe-rs WASM, an empty
 * submodule in the reference; its surface is visible at sdk/relayer/src/tfhe.ts:1-28 and
 * packages/luxfhejs/src/index.ts:42-200):
 *   genKeys / ClientKey / ServerKey   <- TfheClientKey.generate + server key (tfhe.ts:20-28)
 *   Engine.pbs / keyswitchProgrammableBootstrap / generateAccumulator
 *                                      <- ServerKey::keyswitch_programmable_bootstrap (biometrics main.rs:65-71)
 *   FheBool (nand/and/or/xor/not), FheUint8/16/32 bitwise ops
 *   LuxFHELocalClient                  <- LuxFHEClient (luxfhejs) method names, computed locally
 * Every homomorphic operation runs on the GPU through libtfhe_hip.so (N-API, async work);
 * keygen / encrypt / decrypt are the client-side host code of the same library.
 */
const path = require('path');
const native = require(path.join(__dirname, 'build', 'tfhe_napi.node'));

const PRESET_GATE = 0;
const PRESET_FHEVM = 1;
const TORUS = 1n << 64n;
const MU = 1n << 61n; // gate encoding: true = +1/8, false = -1/8

const mod64 = (x) => ((x % TORUS) + TORUS) % TORUS;

function paramsPreset(which = PRESET_GATE) {
  return native.paramsPreset(which);
}

class ClientKey {
  constructor(params, seed, lweKey, glweKey) {
    this.params = params;
    this.seed = BigInt(seed);
    this.lweKey = lweKey;
    this.glweKey = glweKey;
  }
  static generate(params = paramsPreset(), seed = 0x7F4E0001n) {
    const k = native.keygen(params, BigInt(seed), false);
    return new ClientKey(k.params, seed, k.lweKey, k.glweKey);
  }
  get ioKey() { return this.params.order === 0 ? this.lweKey : this.glweKey; }
  get ioNoise() { return this.params.order === 0 ? this.params.lwe_noise_log2 : this.params.glwe_noise_log2; }
  get ctLen() { return this.ioKey.length + 1; }

  encryptTorus(msgs, seed = 1n, stream0 = 0n) {
    const m = msgs instanceof BigUint64Array ? msgs : BigUint64Array.from(msgs, (v) => mod64(BigInt(v)));
    return native.encrypt(this.ioKey, this.ioNoise, BigInt(seed), BigInt(stream0), m);
  }
  phase(cts) { return native.phase(this.ioKey, cts); }

  encryptBool(bits, seed = 1n, stream0 = 0n) {
    return this.encryptTorus(Array.from(bits, (b) => (b ? MU : TORUS - MU)), seed, stream0);
  }
  decryptBool(cts) { return Array.from(this.phase(cts), (p) => p < (1n << 63n)); }

  /** shortint encoding with one padding bit (encryption.rs:5-22) */
  encrypt(values, msgModulus, seed = 1n, stream0 = 0n) {
    const delta = (1n << 63n) / BigInt(msgModulus);
    return this.encryptTorus(Array.from(values, (v) => (BigInt(v) % BigInt(msgModulus)) * delta), seed, stream0);
  }
  decrypt(cts, msgModulus) {
    const delta = (1n << 63n) / BigInt(msgModulus);
    return Array.from(this.phase(cts), (p) => Number(((p + delta / 2n) / delta) % BigInt(msgModulus)));
  }
}

class ServerKey {
  constructor(params, bsk, ksk) { this.params = params; this.bsk = bsk; this.ksk = ksk; }
}

/** tfhe-rs gen_keys analogue: deterministic ChaCha20-seeded key set -> [ClientKey, ServerKey] */
function genKeys(params = paramsPreset(), seed = 0x7F4E0001n) {
  const k = native.keygen(params, BigInt(seed), true);
  return [new ClientKey(k.params, seed, k.lweKey, k.glweKey), new ServerKey(k.params, k.bsk, k.ksk)];
}

class Engine {
  constructor(params = paramsPreset(), device = 0) {
    this.params = params;
    this.handle = native.createEngine(params, device);
  }
  loadKeys(serverKey) { native.loadKeys(this.handle, serverKey.bsk, serverKey.ksk); return this; }
  destroy() { if (this.handle) { native.destroyEngine(this.handle); this.handle = null; } }
  gateLut() { return native.lutConstant(this.params.N, MU); }
  generateAccumulator(f, msgModulus = 4, deltaOut = null) {
    const mm = BigInt(msgModulus);
    const delta = deltaOut === null ? (1n << 63n) / mm : BigInt(deltaOut);
    const table = BigUint64Array.from({ length: msgModulus }, (_, m) => mod64(BigInt(f(m)) % mm));
    return native.lutFromTable(this.params.N, msgModulus, table, delta);
  }
  /** batched PBS (blind rotate + sample extract + keyswitch) on the GPU; resolves to ciphertexts */
  pbs(cts, luts, lutIndex = null) { return native.pbs(this.handle, cts, luts, lutIndex); }
  keyswitchProgrammableBootstrap(ct, acc) { return this.pbs(ct, acc); }
  nand(c1, c2) { return native.nand(this.handle, c1, c2); }
}

/* gate linear part (0, c) + k1*c1 + k2*c2 over Z_2^64, ciphertext-wise */
function gateLin(c1, c2, k1, k2, c, ctLen) {
  const out = new BigUint64Array(c1.length);
  const K1 = mod64(BigInt(k1)), K2 = mod64(BigInt(k2)), C = mod64(BigInt(c));
  for (let i = 0; i < c1.length; i++) {
    let v = c1[i] * K1 + (c2 ? c2[i] * K2 : 0n);
    if ((i + 1) % ctLen === 0) v += C;
    out[i] = mod64(v);
  }
  return out;
}

class FheBool {
  constructor(engine, ct) { this.engine = engine; this.ct = ct; this.ctLen = engine.params.n + 1; }
  static encrypt(values, clientKey, engine, seed = 1n, stream0 = 0n) {
    const arr = Array.isArray(values) ? values : [values];
    return new FheBool(engine, clientKey.encryptBool(arr, seed, stream0));
  }
  decrypt(clientKey) { return clientKey.decryptBool(this.ct); }
  async _boot(lin) { return new FheBool(this.engine, await this.engine.pbs(lin, this.engine.gateLut())); }
  async nand(o) { return new FheBool(this.engine, await this.engine.nand(this.ct, o.ct)); }
  and(o) { return this._boot(gateLin(this.ct, o.ct, 1, 1, -MU, this.ctLen)); }
  or(o) { return this._boot(gateLin(this.ct, o.ct, 1, 1, MU, this.ctLen)); }
  xor(o) { return this._boot(gateLin(this.ct, o.ct, 2, 2, 2n * MU, this.ctLen)); }
  not() { return new FheBool(this.engine, gateLin(this.ct, null, -1, 0, 0, this.ctLen)); }
}

/** FheUintN as N gate-encoded bits (LSB first); bitwise ops bootstrap all bits in one batch. */
function makeUint(bits) {
  return class {
    constructor(engine, ct) { this.engine = engine; this.ct = ct; this.bits = bits; }
    static get bitWidth() { return bits; }
    static encrypt(values, clientKey, engine, seed = 1n, stream0 = 0n) {
      const vs = Array.isArray(values) ? values : [values];
      const flat = [];
      for (const v of vs) for (let j = 0; j < bits; j++) flat.push(((BigInt(v) >> BigInt(j)) & 1n) === 1n);
      return new this(engine, clientKey.encryptBool(flat, seed, stream0));
    }
    decrypt(clientKey) {
      const b = clientKey.decryptBool(this.ct);
      const out = [];
      for (let i = 0; i < b.length; i += bits) {
        let v = 0n;
        for (let j = 0; j < bits; j++) if (b[i + j]) v |= 1n << BigInt(j);
        out.push(v);
      }
      return out;
    }
    _wrap(ct) { return new this.constructor(this.engine, ct); }
    async and(o) { return this._wrap((await new FheBool(this.engine, this.ct).and(new FheBool(this.engine, o.ct))).ct); }
    async or(o) { return this._wrap((await new FheBool(this.engine, this.ct).or(new FheBool(this.engine, o.ct))).ct); }
    async xor(o) { return this._wrap((await new FheBool(this.engine, this.ct).xor(new FheBool(this.engine, o.ct))).ct); }
    not() { return this._wrap(new FheBool(this.engine, this.ct).not().ct); }
  };
}
const FheUint8 = makeUint(8);
const FheUint16 = makeUint(16);
const FheUint32 = makeUint(32);

/**
 * LuxFHEClient-compatible local client (packages/luxfhejs/src/index.ts:42-200 method names).
 * encrypt_* return the serialized ciphertext bytes (Uint8Array) like the HTTP client; evaluate()
 * covers the bitwise ops of POST /evaluate (e2e/test/fhe.test.ts:105-175) on the GPU.
 */
class LuxFHELocalClient {
  constructor(config = {}) {
    this.params = config.params || paramsPreset(PRESET_GATE);
    this.seed = BigInt(config.seed || 0x7F4E0001n);
    this.device = config.device || 0;
    this.engine = null;
    this.clientKey = null;
    this.serverKey = null;
    this.stream = 0n;
  }
  async initialize() {
    [this.clientKey, this.serverKey] = genKeys(this.params, this.seed);
    this.engine = new Engine(this.params, this.device).loadKeys(this.serverKey);
  }
  async getPublicKey() {
    // this scheme's evaluation key = BSK || KSK (standard domain, u64 LE)
    const b = this.serverKey.bsk, k = this.serverKey.ksk;
    const out = new Uint8Array((b.length + k.length) * 8);
    out.set(new Uint8Array(b.buffer, b.byteOffset, b.byteLength), 0);
    out.set(new Uint8Array(k.buffer, k.byteOffset, k.byteLength), b.byteLength);
    return out;
  }
  _enc(value, bitWidth) {
    const cls = { 8: FheUint8, 16: FheUint16, 32: FheUint32 }[bitWidth];
    if (!cls) throw new Error(`Encryption failed: bitWidth ${bitWidth} not supported by the local engine`);
    const ct = cls.encrypt([value], this.clientKey, this.engine, this.seed + 1n, this.stream).ct;
    this.stream += BigInt(bitWidth);
    return new Uint8Array(ct.buffer, ct.byteOffset, ct.byteLength);
  }
  async encrypt_uint8(v) { return this._enc(v, 8); }
  async encrypt_uint16(v) { return this._enc(v, 16); }
  async encrypt_uint32(v) { return this._enc(v, 32); }
  _ct(bytes) { return new BigUint64Array(bytes.buffer.slice(bytes.byteOffset, bytes.byteOffset + bytes.byteLength)); }
  async evaluate({ op, left, right, bitWidth }) {
    const cls = { 8: FheUint8, 16: FheUint16, 32: FheUint32 }[bitWidth];
    const a = new cls(this.engine, this._ct(left));
    const b = right ? new cls(this.engine, this._ct(right)) : null;
    let r;
    if (op === 'and') r = await a.and(b);
    else if (op === 'or') r = await a.or(b);
    else if (op === 'xor') r = await a.xor(b);
    else if (op === 'not') r = a.not();
    else throw new Error(`evaluate: op ${op} not supported by the local engine`);
    return new Uint8Array(r.ct.buffer, r.ct.byteOffset, r.ct.byteLength);
  }
  async decrypt(bytes, bitWidth) {
    const cls = { 8: FheUint8, 16: FheUint16, 32: FheUint32 }[bitWidth];
    return new cls(this.engine, this._ct(bytes)).decrypt(this.clientKey)[0];
  }
  close() { if (this.engine) this.engine.destroy(); }
}

module.exports = {
  native, PRESET_GATE, PRESET_FHEVM, MU, paramsPreset, genKeys, ClientKey, ServerKey, Engine,
  FheBool, FheUint8, FheUint16, FheUint32, LuxFHELocalClient,
};
