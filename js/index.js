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
 *   FheBool (nand/and/or/xor/not), FheUint8..256 with every fhEVM operator (js/integer.js)
 *   LuxFHELocalClient                  <- LuxFHEClient (luxfhejs) method names, computed locally
 * Every homomorphic operation runs on the GPU through libtfhe_hip.so (N-API, async work);
 * keygen / encrypt / decrypt are the client-side host code of the same library.
 */
const path = require('path');
const native = require(path.join(__dirname, 'build', 'tfhe_napi.node'));
const integer = require('./integer.js');
const radix = require('./radix.js');

const PRESET_GATE = 0;
const PRESET_FHEVM = 1;
const PRESET_GATE_FFT = 2;  // P-GATE on the FFT64 transform (tfhe-rs's f64-FFT external product)
const PRESET_FHEVM_FFT = 3; // P-FHEVM on the FFT64 transform
const TORUS = 1n << 64n;
const MU = 1n << 61n; // gate encoding: true = +1/8, false = -1/8

const mod64 = (x) => ((x % TORUS) + TORUS) % TORUS;

function paramsPreset(which = PRESET_GATE) {
  return native.paramsPreset(which);
}

class ClientKey {
  /** seed: the test seed the keys came from, or null for keys drawn from OS entropy */
  constructor(params, seed, lweKey, glweKey) {
    this.params = params;
    this.seed = seed === undefined || seed === null ? null : BigInt(seed);
    this.lweKey = lweKey;
    this.glweKey = glweKey;
  }
  /** seed undefined (default): 192-bit OS entropy; a seed: the reproducible TEST key (public knowledge) */
  static generate(params = paramsPreset(), seed = undefined) {
    const k = native.keygen(params, rngArg(seed), false);
    return new ClientKey(k.params, seed, k.lweKey, k.glweKey);
  }
  get ioKey() { return this.params.order === 0 ? this.lweKey : this.glweKey; }
  get ioNoise() { return this.params.order === 0 ? this.params.lwe_noise_log2 : this.params.glwe_noise_log2; }
  get ctLen() { return this.ioKey.length + 1; }

  /** seed undefined (default): masks and noise from a fresh OS-entropy ChaCha key for this call */
  encryptTorus(msgs, seed = undefined, stream0 = 0n) {
    const m = msgs instanceof BigUint64Array ? msgs : BigUint64Array.from(msgs, (v) => mod64(BigInt(v)));
    return native.encrypt(this.ioKey, this.ioNoise, rngArg(seed), BigInt(stream0), m);
  }
  phase(cts) { return native.phase(this.ioKey, cts); }

  encryptBool(bits, seed = undefined, stream0 = 0n) {
    return this.encryptTorus(Array.from(bits, (b) => (b ? MU : TORUS - MU)), seed, stream0);
  }
  decryptBool(cts) { return Array.from(this.phase(cts), (p) => p < (1n << 63n)); }

  /** shortint encoding with one padding bit (encryption.rs:5-22) */
  encrypt(values, msgModulus, seed = undefined, stream0 = 0n) {
    const delta = (1n << 63n) / BigInt(msgModulus);
    return this.encryptTorus(Array.from(values, (v) => (BigInt(v) % BigInt(msgModulus)) * delta), seed, stream0);
  }
  decrypt(cts, msgModulus) {
    const delta = (1n << 63n) / BigInt(msgModulus);
    return Array.from(this.phase(cts), (p) => Number(((p + delta / 2n) / delta) % BigInt(msgModulus)));
  }
}

class ServerKey {
  // msZeros: P-FHEVM modulus-switch noise-reduction zeros (KS -> PBS parameter sets only)
  constructor(params, bsk, ksk, msZeros = null) { this.params = params; this.bsk = bsk; this.ksk = ksk; this.msZeros = msZeros; }
}

/** undefined -> OS entropy (native side); a seed -> the reproducible test stream */
const rngArg = (seed) => (seed === undefined || seed === null ? undefined : BigInt(seed));

/** tfhe-rs gen_keys analogue -> [ClientKey, ServerKey].  seed undefined (default): every key from 192 bits
 *  of OS entropy; a seed gives the reproducible TEST key set (anyone knowing it can decrypt). */
function genKeys(params = paramsPreset(), seed = undefined) {
  const k = native.keygen(params, rngArg(seed), true);
  return [new ClientKey(k.params, seed, k.lweKey, k.glweKey), new ServerKey(k.params, k.bsk, k.ksk, k.msZeros || null)];
}

/** devices: one GPU ordinal or an array (one shard each; batches split across them, keys broadcast once
 *  over RCCL -- include/tfhe_hip.h tfhe_hip_create) */
class Engine {
  constructor(params = paramsPreset(), devices = 0) {
    this.params = params;
    this.handle = native.createEngine(params, devices);
  }
  info() { return native.engineInfo(this.handle); }
  loadKeys(serverKey) { native.loadKeys(this.handle, serverKey.bsk, serverKey.ksk, serverKey.msZeros || null); return this; }
  destroy() { if (this.handle) { native.destroyEngine(this.handle); this.handle = null; } }
  gateLut() { return native.lutConstant(this.params.N, MU); }
  generateAccumulator(f, msgModulus = 4, deltaOut = null) {
    const mm = BigInt(msgModulus);
    const delta = deltaOut === null ? (1n << 63n) / mm : BigInt(deltaOut);
    const table = BigUint64Array.from({ length: msgModulus }, (_, m) => mod64(BigInt(f(m)) % mm));
    return native.lutFromTable(this.params.N, msgModulus, table, delta);
  }
  /** LUT for a lookup table of msgModulus entries (radix blocks: 16 = message x carry, padding bit kept) */
  lutFromTable(table, msgModulus = table.length) {
    const t = BigUint64Array.from(table, (v) => BigInt(v));
    return native.lutFromTable(this.params.N, msgModulus, t, (1n << 63n) / BigInt(msgModulus));
  }
  /** batched PBS (blind rotate + sample extract + keyswitch) on the GPU; resolves to ciphertexts */
  pbs(cts, luts, lutIndex = null) { return native.pbs(this.handle, cts, luts, lutIndex); }
  keyswitchProgrammableBootstrap(ct, acc) { return this.pbs(ct, acc); }
  /** LWE keyswitch B x (kN+1) -> B x (n+1) (the KS stage alone); resolves to ciphertexts */
  keyswitch(bigLwes) { return native.keyswitch(this.handle, bigLwes); }
  /** blind rotation of small-key LWEs B x (n+1) -> B x (k+1) x N accumulators (stage-level) */
  blindRotate(cts, luts, lutIndex = null) { return native.blindRotate(this.handle, cts, luts, lutIndex); }
  nand(c1, c2) { return native.nand(this.handle, c1, c2); }
}

/**
 * Ciphertext compression (ml/extensions/rust/src/compression.rs:222,276: LWE list -> GLWE packing keyswitch, then
 * CompressedModulusSwitchedGlweCiphertext::compress) on the GPU.  PARAMS_8B_2048_NEW: LWE dim 2048 -> k = 1,
 * N = 2048, 2 x 2^14, 2048 LWEs per GLWE, 26-bit storage.
 */
class Packer {
  constructor(device = 0) { this.handle = native.createPacker(device); }
  /** inKey: the LWE key of the inputs (BigUint64Array(2048) bits); seed undefined = OS entropy.
   *  -> {outKey (client, decrypts the packed GLWEs), pksk (server)} */
  static keygen(inKey, seed = undefined) { return native.pksKeygen(inKey, rngArg(seed)); }
  loadKey(pksk) { native.loadAuxKey(this.handle, pksk); return this; }
  /** lwes: count x 2049 -> Promise<[{glwe, packed, bodies}]> one entry per GLWE of up to 2048 LWEs */
  async packCompress(lwes) {
    const r = await native.packCompress(this.handle, lwes);
    const glweLen = 2 * 2048, count = lwes.length / 2049, out = [];
    let off = 0;
    for (let g = 0; g * 2048 < count; g++) {
      const bodies = Math.min(2048, count - g * 2048);
      const words = Math.ceil((2048 + bodies) * 26 / 64);   // tfhe_hip_pks_packed_words: 26 bits per coefficient
      out.push({ glwe: r.glwes.subarray(g * glweLen, (g + 1) * glweLen), packed: r.packed.subarray(off, off + words), bodies });
      off += words;
    }
    if (off !== r.packed.length) throw new Error(`packCompress: ${off} packed words expected, ${r.packed.length} returned`);
    return out;
  }
  /** the decompression of one compressed GLWE (host) */
  static extract(packed, bodies) { return native.extractGlwe(packed, bodies); }
  static glwePhase(key, glwe) { return native.glwePhase(key, glwe); }
  destroy() { if (this.handle) { native.destroyAux(this.handle); this.handle = null; } }
}

/**
 * Switch-and-squash noise squashing (the fhEVM sns-worker, tests/fhevm-suite/fhevm/docker-compose/
 * coprocessor-docker-compose.yml:124-140): P-FHEVM ciphertexts -> 128-bit LWEs (k = 2, N = 2048 squashing key)
 * with ~2^-63 noise for threshold decryption.
 */
class Squasher {
  constructor(device = 0) { this.handle = native.createSquasher(device); }
  /** lweKey: the P-FHEVM small LWE key (918 bits); -> {glweKey (client, 128-bit), bsk (server)} */
  static keygen(lweKey, seed = undefined) { return native.snsKeygen(lweKey, rngArg(seed)); }
  loadKey(bsk) { native.loadAuxKey(this.handle, bsk); return this; }
  /** engine: the P-FHEVM Engine holding the server key (keyswitch + modulus-switch reduction);
   *  cts: B x 2049 -> Promise<BigUint64Array> B x 4097 x 2 ((lo, hi) words of the 128-bit LWEs) */
  squash(engine, cts, msgModulus = 16) { return native.squash(this.handle, engine.handle, cts, msgModulus); }
  /** client side: decrypt squashed ciphertexts (one padding bit, msgModulus values) */
  static decrypt(glweKey, cts, msgModulus = 16) {
    const ph = native.snsPhase(glweKey, cts), out = [];
    const delta = (1n << 127n) / BigInt(msgModulus);
    for (let i = 0; i < ph.length; i += 2) {
      const v = ph[i] | (ph[i + 1] << 64n);
      out.push(Number(((v + delta / 2n) / delta) % BigInt(msgModulus)));
    }
    return out;
  }
  destroy() { if (this.handle) { native.destroyAux(this.handle); this.handle = null; } }
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
  static encrypt(values, clientKey, engine, seed = undefined, stream0 = 0n) {
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

/**
 * Ciphertext bytes (the opaque Uint8Array of the HTTP API and LuxFHEClient): a 16-byte header
 *   'TFA1' | u8 kind | u8 0 | u16 width | u32 lwe_dim | u32 count
 * then count x cts(kind, width) x (lwe_dim + 1) u64 little-endian (value-major, LSB first).
 * kind 0 = ebool, 1 = euint (one gate ciphertext per bit, P-GATE); kind 2 = radix euint (width/2
 * blocks of 2 message bits, P-FHEVM), 3 = radix ebool (one block holding 0/1).
 */
const CT_MAGIC = 0x31414654; // 'TFA1'
const KIND = { BOOL: 0, UINT: 1, RADIX_UINT: 2, RADIX_BOOL: 3 };
const ctsPerValue = (kind, width) => (kind === KIND.RADIX_UINT ? width / 2 : kind === KIND.RADIX_BOOL ? 1 : width);
function serializeCiphertext(kind, width, lweDim, count, words) {
  const out = new Uint8Array(16 + words.byteLength);
  const dv = new DataView(out.buffer);
  dv.setUint32(0, CT_MAGIC, true);
  dv.setUint8(4, kind);
  dv.setUint16(6, width, true);
  dv.setUint32(8, lweDim, true);
  dv.setUint32(12, count, true);
  out.set(new Uint8Array(words.buffer, words.byteOffset, words.byteLength), 16);
  return out;
}
function parseCiphertext(bytes) {
  const u8 = bytes instanceof Uint8Array ? bytes : Uint8Array.from(bytes);
  if (u8.length < 16) throw new Error('ciphertext too short');
  const dv = new DataView(u8.buffer, u8.byteOffset, u8.byteLength);
  if (dv.getUint32(0, true) !== CT_MAGIC) throw new Error('not a tfhe_amd ciphertext (bad magic)');
  const kind = dv.getUint8(4), width = dv.getUint16(6, true), lweDim = dv.getUint32(8, true), count = dv.getUint32(12, true);
  if (kind > 3 || (kind === KIND.RADIX_UINT && width % 2)) throw new Error(`bad ciphertext kind ${kind} / width ${width}`);
  const nWords = count * ctsPerValue(kind, width) * (lweDim + 1);
  if (u8.length !== 16 + 8 * nWords) throw new Error(`ciphertext length ${u8.length} != header size ${16 + 8 * nWords}`);
  const words = new BigUint64Array(u8.buffer.slice(u8.byteOffset + 16, u8.byteOffset + u8.byteLength));
  return { kind, width, lweDim, count, words };
}

/** FheUintN: a batch of N-bit encrypted integers over gate bootstrapping (js/integer.js). */
function makeUint(bits) {
  return class {
    constructor(engine, ct, count = null) {
      this.engine = engine;
      this.ct = ct; // value-major [count][bits][n+1]
      this.bits = bits;
      this.count = count === null ? ct.length / (bits * (engine.params.n + 1)) : count;
    }
    static get bitWidth() { return bits; }
    static encrypt(values, clientKey, engine, seed = undefined, stream0 = 0n) {
      const vs = Array.isArray(values) ? values : [values];
      const flat = [];
      for (const v of vs) for (let j = 0; j < bits; j++) flat.push(((BigInt(v) >> BigInt(j)) & 1n) === 1n);
      return new this(engine, clientKey.encryptBool(flat, seed, stream0), vs.length);
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
    _vec(circuit) { return integer.FheUintVec.fromValueMajor(circuit, this.ct, this.count, bits); }
    /** any fhEVM operator (js/integer.js); other: FheUint* of any width or a plaintext */
    async op(name, other = null) {
      const c = new integer.Circuit(this.engine);
      const rhs = other && other.ct ? other._vec(c) : other;
      const r = await c.run(integer.fhevmOp(c, name, this._vec(c), rhs));
      if (r instanceof integer.FheUintVec) return new (UINT_CLASSES[r.width] || makeUint(r.width))(this.engine, r.toValueMajor(), r.B);
      return new FheBool(this.engine, r);
    }
    and(o) { return this.op('and', o); }
    or(o) { return this.op('or', o); }
    xor(o) { return this.op('xor', o); }
    not() { return new this.constructor(this.engine, gateLin(this.ct, null, -1, 0, 0, this.engine.params.n + 1), this.count); }
    add(o) { return this.op('add', o); }
    sub(o) { return this.op('sub', o); }
    mul(o) { return this.op('mul', o); }
    eq(o) { return this.op('eq', o); }
    ne(o) { return this.op('ne', o); }
    lt(o) { return this.op('lt', o); }
    le(o) { return this.op('le', o); }
    gt(o) { return this.op('gt', o); }
    ge(o) { return this.op('ge', o); }
    min(o) { return this.op('min', o); }
    max(o) { return this.op('max', o); }
  };
}
const UINT_CLASSES = {};
for (const w of [8, 16, 32, 64, 128, 160, 256]) UINT_CLASSES[w] = makeUint(w);
const FheUint8 = UINT_CLASSES[8];
const FheUint16 = UINT_CLASSES[16];
const FheUint32 = UINT_CLASSES[32];
const FheUint64 = UINT_CLASSES[64];

/**
 * LuxFHEClient-compatible local client (packages/luxfhejs/src/index.ts:42-200 method names).
 * encrypt_* return serialized ciphertext bytes (Uint8Array) like the HTTP client; evaluate() takes
 * the POST /evaluate shape (e2e/test/fhe.test.ts:105-175) and runs every fhEVM operator on the GPU.
 * Requests submitted concurrently are evaluated in lockstep (one PBS launch per circuit level).
 * config.params: a params object, or 'gate_fft' (default: boolean gates on the FFT64 transform -- the
 * engine the bench measures -- js/integer.js), 'fhevm_fft' (P-FHEVM radix blocks, js/radix.js, fhEVM's
 * own representation), or 'gate' / 'fhevm' for the same parameter sets on the Goldilocks NTT transform.
 * config.devices: a GPU ordinal or an array of ordinals (batches split across them, keys broadcast once).
 * Keys and every encryption draw fresh OS entropy.  config.seed (a reproducible, PUBLIC key set: anyone
 * who knows it decrypts everything) is refused unless config.dev is true.
 */
class LuxFHELocalClient {
  constructor(config = {}) {
    const pr = config.params;
    const named = { gate: PRESET_GATE, fhevm: PRESET_FHEVM, gate_fft: PRESET_GATE_FFT, fhevm_fft: PRESET_FHEVM_FFT };
    if (typeof pr === 'string' && !(pr in named)) throw new Error(`unknown params preset '${pr}'`);
    this.params = !pr ? paramsPreset(PRESET_GATE_FFT) : typeof pr === 'string' ? paramsPreset(named[pr]) : pr;
    this.radix = this.params.order === 1;
    this.dim = this.radix ? this.params.k * this.params.N : this.params.n;
    if (config.seed !== undefined && config.seed !== null && !config.dev)
      throw new Error('LuxFHELocalClient: a fixed seed makes every key and ciphertext reproducible by anyone who '
                      + 'knows it; pass {dev: true} to use one (tests / demos only)');
    this.seed = config.seed === undefined || config.seed === null ? null : BigInt(config.seed);
    this.devices = config.devices !== undefined ? config.devices : (config.device || 0);
    this.engine = config.engine || null;
    this.clientKey = null;
    this.serverKey = null;
    this.stream = 0n;
    this.queue = [];
    this.busy = false;
    this.launches = 0;
  }
  async initialize() {
    [this.clientKey, this.serverKey] = genKeys(this.params, this.seed === null ? undefined : this.seed);
    if (!this.engine) this.engine = new Engine(this.params, this.devices).loadKeys(this.serverKey);
  }
  /** key descriptor: params + SHA-256 of the evaluation keys (this scheme has no public encryption key) */
  async getPublicKey() {
    const crypto = require('crypto');
    const h = crypto.createHash('sha256');
    for (const a of [this.serverKey.bsk, this.serverKey.ksk]) h.update(new Uint8Array(a.buffer, a.byteOffset, a.byteLength));
    const p = this.params;
    const head = new Uint32Array([0x314B4654, p.n, p.k, p.N, p.pbs_base_log, p.pbs_level, p.ks_base_log, p.ks_level, p.order]);
    const out = new Uint8Array(head.byteLength + 32);
    out.set(new Uint8Array(head.buffer), 0);
    out.set(h.digest(), head.byteLength);
    return out;
  }
  /** dev seed: the reproducible stream seed+1 (stream counter advances); otherwise undefined = fresh
   *  OS entropy for every encryption, so no two ciphertexts share masks or noise, across restarts too */
  _encSeed() { return this.seed === null ? undefined : this.seed + 1n; }
  encryptValue(value, bitWidth) {
    const w = Number(bitWidth);
    if (!(w >= 1 && w <= 256)) throw new Error(`Encryption failed: bitWidth ${bitWidth} not supported`);
    const v = BigInt.asUintN(w, BigInt(value));
    if (this.radix) {
      if (w > 1 && w % 2) throw new Error(`Encryption failed: radix bitWidth ${w} must be even`);
      const nb = w === 1 ? 1 : w / 2;
      const digits = Array.from({ length: nb }, (_, j) => (v >> BigInt(2 * j)) & 3n);
      const ct = this.clientKey.encrypt(digits, radix.SPACE, this._encSeed(), this.stream);
      this.stream += BigInt(nb);
      return serializeCiphertext(w === 1 ? KIND.RADIX_BOOL : KIND.RADIX_UINT, w, this.dim, 1, ct);
    }
    const flat = [];
    for (let j = 0; j < w; j++) flat.push(((v >> BigInt(j)) & 1n) === 1n);
    const ct = this.clientKey.encryptBool(flat, this._encSeed(), this.stream);
    this.stream += BigInt(w);
    return serializeCiphertext(w === 1 ? 0 : 1, w, this.params.n, 1, ct);
  }
  async encrypt_bool(v) { return this.encryptValue(v ? 1 : 0, 1); }
  async encrypt_uint8(v) { return this.encryptValue(v, 8); }
  async encrypt_uint16(v) { return this.encryptValue(v, 16); }
  async encrypt_uint32(v) { return this.encryptValue(v, 32); }
  async encrypt_uint64(v) { return this.encryptValue(v, 64); }
  async encrypt_uint128(v) { return this.encryptValue(v, 128); }
  async encrypt_uint256(v) { return this.encryptValue(v, 256); }
  async encrypt_address(a) { return this.encryptValue(BigInt(a), 160); }

  _operand(x, bitWidth, circuit) {
    if (x === null || x === undefined) return null;
    if (typeof x === 'number' || typeof x === 'bigint' || typeof x === 'string') return BigInt(x);
    const ct = parseCiphertext(x);
    if (ct.lweDim !== this.dim) throw new Error(`ciphertext lwe_dim ${ct.lweDim} != engine ${this.dim}`);
    if (this.radix !== (ct.kind >= KIND.RADIX_UINT)) throw new Error(`ciphertext kind ${ct.kind} does not match the engine parameters`);
    if (this.radix) return radix.RadixVec.fromValueMajor(circuit, ct.words, ct.count, ctsPerValue(ct.kind, ct.width));
    return integer.FheUintVec.fromValueMajor(circuit, ct.words, ct.count, ct.width);
  }
  _radixGen(c, op, l, r) {
    // ebool operands are one-block radix values holding 0/1; logical not is 1 - x on them
    if (op === 'not' && l.blocks.length === 1 && l.isBool) {
      const one = c.const(l.B, 1);
      for (let i = 0; i < one.length; i++) one[i] = BigInt.asUintN(64, one[i] - l.blocks[0][i]);
      return (function* () { return one; }());
    }
    return radix.fhevmOp(c, op, l, r);
  }
  /** POST /evaluate: { op, left, right?, bitWidth } -> ciphertext bytes (ebool for comparisons) */
  evaluate(req) {
    return new Promise((resolve, reject) => {
      this.queue.push({ req, resolve, reject });
      this._pump();
    });
  }
  async _pump() {
    if (this.busy || !this.queue.length) return;
    this.busy = true;
    const jobs = this.queue.splice(0);
    const c = this.radix ? new radix.RadixCircuit(this.engine) : new integer.Circuit(this.engine);
    const live = [];
    for (const j of jobs) {
      try {
        const { op, left, right } = j.req;
        const l = this._operand(left, j.req.bitWidth, c), r = this._operand(right, j.req.bitWidth, c);
        if (this.radix) {
          const isB = (x) => x !== null && x !== undefined && typeof x === 'object' && parseCiphertext(x).kind === KIND.RADIX_BOOL;
          l.isBool = isB(left);
          if (r instanceof radix.RadixVec) r.isBool = isB(right);
          live.push({ j, gen: this._radixGen(c, op, l, r), bool: l.isBool && (!(r instanceof radix.RadixVec) || r.isBool) });
        } else {
          live.push({ j, gen: integer.fhevmOp(c, op, l, r) });
        }
      } catch (e) { j.reject(e); }
    }
    try {
      const res = await c.runMany(live.map((x) => x.gen));
      this.launches += c.launches;
      const d = this.dim + 1;
      res.forEach((r, i) => {
        if (r instanceof integer.FheUintVec) live[i].j.resolve(serializeCiphertext(KIND.UINT, r.width, this.dim, r.B, r.toValueMajor()));
        else if (r instanceof radix.RadixVec) {
          // and/or/xor on ebool operands stay ebool (one block)
          if (live[i].bool && r.blocks.length === 1) live[i].j.resolve(serializeCiphertext(KIND.RADIX_BOOL, 1, this.dim, r.B, r.toValueMajor()));
          else live[i].j.resolve(serializeCiphertext(KIND.RADIX_UINT, r.width, this.dim, r.B, r.toValueMajor()));
        } else live[i].j.resolve(serializeCiphertext(this.radix ? KIND.RADIX_BOOL : KIND.BOOL, 1, this.dim, r.length / d, r));
      });
    } catch (e) {
      live.forEach((x) => x.j.reject(e));
    }
    this.busy = false;
    this._pump();
  }
  /** -> bigint (first value of the ciphertext); decryption is host-side, so this is synchronous */
  decryptSync(bytes) {
    const ct = parseCiphertext(bytes);
    const c = { dim: ct.lweDim + 1 };
    if (ct.kind >= KIND.RADIX_UINT) {
      const vec = radix.RadixVec.fromValueMajor(c, ct.words, ct.count, ctsPerValue(ct.kind, ct.width));
      return radix.decryptRadix(this.clientKey, vec)[0];
    }
    const vec = integer.FheUintVec.fromValueMajor(c, ct.words, ct.count, ct.width);
    return integer.decryptColumns(this.clientKey, vec.cols, ct.count)[0];
  }
  async decrypt(bytes) { return this.decryptSync(bytes); }
  /**
   * luxfhejs unseal(contractAddress, sealedData): bigint -- synchronous like the reference
   * (packages/luxfhejs/src/index.ts:146); sealedData as bytes or a hex string ("0x..." or bare hex)
   */
  unseal(_addr, data) {
    if (typeof data === 'string') {
      const h = data.startsWith('0x') || data.startsWith('0X') ? data.slice(2) : data;
      if (h.length % 2 !== 0 || /[^0-9a-fA-F]/.test(h)) throw new Error('unseal: sealedData is not a hex string');
      data = Uint8Array.from(Buffer.from(h, 'hex'));
    }
    return this.decryptSync(data);
  }
  close() { if (this.engine && this.engine.destroy) this.engine.destroy(); }
}

module.exports = {
  native, integer, radix, KIND, PRESET_GATE, PRESET_FHEVM, PRESET_GATE_FFT, PRESET_FHEVM_FFT, MU, paramsPreset, genKeys, ClientKey, ServerKey, Engine,
  Packer, Squasher, FheBool, FheUint8, FheUint16, FheUint32, FheUint64, UINT_CLASSES, LuxFHELocalClient,
  serializeCiphertext, parseCiphertext,
};
