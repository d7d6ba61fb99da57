// Type declarations for @luxfhe-amd/tfhe (js/index.js).  Mirrors the FheBool / FheUint* and
// LuxFHEClient surfaces of the reference (packages/luxfhejs/src/index.ts, sdk/relayer/src/tfhe.ts).
export interface TfheParams {
  n: number; k: number; N: number; pbs_base_log: number; pbs_level: number;
  ks_base_log: number; ks_level: number; lwe_noise_log2: number; glwe_noise_log2: number; order: number;
}
export const PRESET_GATE: 0;
export const PRESET_FHEVM: 1;
export const PRESET_GATE_FFT: 2;
export const PRESET_FHEVM_FFT: 3;
export const MU: bigint;
export function paramsPreset(which?: number): TfheParams;

export class ClientKey {
  readonly params: TfheParams; readonly seed: bigint;
  readonly lweKey: BigUint64Array; readonly glweKey: BigUint64Array;
  static generate(params?: TfheParams, seed?: bigint): ClientKey;
  encryptTorus(msgs: BigUint64Array | Iterable<bigint | number>, seed?: bigint, stream0?: bigint): BigUint64Array;
  phase(cts: BigUint64Array): BigUint64Array;
  encryptBool(bits: Iterable<boolean>, seed?: bigint, stream0?: bigint): BigUint64Array;
  decryptBool(cts: BigUint64Array): boolean[];
  encrypt(values: Iterable<number | bigint>, msgModulus: number, seed?: bigint, stream0?: bigint): BigUint64Array;
  decrypt(cts: BigUint64Array, msgModulus: number): number[];
}
export class ServerKey { readonly params: TfheParams; readonly bsk: BigUint64Array; readonly ksk: BigUint64Array; readonly msZeros: BigUint64Array | null; }
export function genKeys(params?: TfheParams, seed?: bigint): [ClientKey, ServerKey];

export class Engine {
  constructor(params?: TfheParams, device?: number);
  loadKeys(sk: ServerKey): this;
  destroy(): void;
  gateLut(): BigUint64Array;
  generateAccumulator(f: (m: number) => number | bigint, msgModulus?: number, deltaOut?: bigint | null): BigUint64Array;
  lutFromTable(table: ArrayLike<number | bigint>, msgModulus?: number): BigUint64Array;
  pbs(cts: BigUint64Array, luts: BigUint64Array, lutIndex?: Uint32Array | null): Promise<BigUint64Array>;
  keyswitchProgrammableBootstrap(ct: BigUint64Array, acc: BigUint64Array): Promise<BigUint64Array>;
  nand(c1: BigUint64Array, c2: BigUint64Array): Promise<BigUint64Array>;
}

export class FheBool {
  constructor(engine: Engine, ct: BigUint64Array);
  readonly ct: BigUint64Array;
  static encrypt(values: boolean | boolean[], ck: ClientKey, engine: Engine, seed?: bigint, stream0?: bigint): FheBool;
  decrypt(ck: ClientKey): boolean[];
  nand(o: FheBool): Promise<FheBool>;
  and(o: FheBool): Promise<FheBool>;
  or(o: FheBool): Promise<FheBool>;
  xor(o: FheBool): Promise<FheBool>;
  not(): FheBool;
}
export type FheOp = 'add' | 'sub' | 'mul' | 'div' | 'rem' | 'and' | 'or' | 'xor' | 'shl' | 'shr' | 'rotl' | 'rotr'
  | 'eq' | 'ne' | 'ge' | 'gt' | 'le' | 'lt' | 'min' | 'max' | 'neg' | 'not';
declare class FheUintN {
  constructor(engine: Engine, ct: BigUint64Array, count?: number);
  readonly ct: BigUint64Array;   // value-major [count][bits][n+1]
  readonly count: number;
  static readonly bitWidth: number;
  decrypt(ck: ClientKey): bigint[];
  /** any fhEVM operator (js/integer.js); comparisons resolve to FheBool */
  op(name: FheOp, other?: FheUintN | number | bigint | null): Promise<FheUintN | FheBool>;
  and(o: FheUintN | bigint): Promise<FheUintN>;
  or(o: FheUintN | bigint): Promise<FheUintN>;
  xor(o: FheUintN | bigint): Promise<FheUintN>;
  not(): FheUintN;
  add(o: FheUintN | bigint): Promise<FheUintN>;
  sub(o: FheUintN | bigint): Promise<FheUintN>;
  mul(o: FheUintN | bigint): Promise<FheUintN>;
  eq(o: FheUintN | bigint): Promise<FheBool>;
  ne(o: FheUintN | bigint): Promise<FheBool>;
  lt(o: FheUintN | bigint): Promise<FheBool>;
  le(o: FheUintN | bigint): Promise<FheBool>;
  gt(o: FheUintN | bigint): Promise<FheBool>;
  ge(o: FheUintN | bigint): Promise<FheBool>;
  min(o: FheUintN | bigint): Promise<FheUintN>;
  max(o: FheUintN | bigint): Promise<FheUintN>;
}
export class FheUint8 extends FheUintN { static encrypt(v: number | bigint | Array<number | bigint>, ck: ClientKey, e: Engine, seed?: bigint, stream0?: bigint): FheUint8; }
export class FheUint16 extends FheUintN { static encrypt(v: number | bigint | Array<number | bigint>, ck: ClientKey, e: Engine, seed?: bigint, stream0?: bigint): FheUint16; }
export class FheUint32 extends FheUintN { static encrypt(v: number | bigint | Array<number | bigint>, ck: ClientKey, e: Engine, seed?: bigint, stream0?: bigint): FheUint32; }
export class FheUint64 extends FheUintN { static encrypt(v: number | bigint | Array<number | bigint>, ck: ClientKey, e: Engine, seed?: bigint, stream0?: bigint): FheUint64; }

/** ciphertext compression (compression.rs:222,276): LWE list -> GLWE packing keyswitch + 26-bit bit packing */
export class Packer {
  constructor(device?: number);
  static keygen(inKey: BigUint64Array, seed?: bigint): { outKey: BigUint64Array; pksk: BigUint64Array };
  loadKey(pksk: BigUint64Array): this;
  packCompress(lwes: BigUint64Array): Promise<Array<{ glwe: BigUint64Array; packed: BigUint64Array; bodies: number }>>;
  static extract(packed: BigUint64Array, bodies: number): BigUint64Array;
  static glwePhase(key: BigUint64Array, glwe: BigUint64Array): BigUint64Array;
  destroy(): void;
}
/** switch-and-squash (the fhEVM sns-worker): P-FHEVM ciphertexts -> 128-bit LWEs, (lo, hi) u64 pairs */
export class Squasher {
  constructor(device?: number);
  static keygen(lweKey: BigUint64Array, seed?: bigint): { glweKey: BigUint64Array; bsk: BigUint64Array };
  loadKey(bsk: BigUint64Array): this;
  squash(engine: Engine, cts: BigUint64Array, msgModulus?: number): Promise<BigUint64Array>;
  static decrypt(glweKey: BigUint64Array, cts: BigUint64Array, msgModulus?: number): number[];
  destroy(): void;
}

/** ciphertext bytes: 'TFA1' | u8 kind | u8 0 | u16 width | u32 lwe_dim | u32 count | u64[] (LE) */
/** kind: 0 ebool / 1 euint (P-GATE bits), 2 radix euint / 3 radix ebool (P-FHEVM blocks) */
export function serializeCiphertext(kind: 0 | 1 | 2 | 3, width: number, lweDim: number, count: number, words: BigUint64Array): Uint8Array;
export function parseCiphertext(bytes: Uint8Array | number[]): { kind: number; width: number; lweDim: number; count: number; words: BigUint64Array };

export interface EvaluateRequest { op: FheOp; left: Uint8Array; right?: Uint8Array | number | bigint | null; bitWidth?: number; }
export class LuxFHELocalClient {
  constructor(config?: { params?: TfheParams | 'gate' | 'fhevm'; seed?: bigint; device?: number; engine?: Engine });
  readonly radix: boolean;
  initialize(): Promise<void>;
  getPublicKey(): Promise<Uint8Array>;
  encryptValue(value: number | bigint | string, bitWidth: number): Uint8Array;
  encrypt_bool(v: boolean): Promise<Uint8Array>;
  encrypt_uint8(v: number | bigint): Promise<Uint8Array>;
  encrypt_uint16(v: number | bigint): Promise<Uint8Array>;
  encrypt_uint32(v: number | bigint): Promise<Uint8Array>;
  encrypt_uint64(v: number | bigint): Promise<Uint8Array>;
  encrypt_uint128(v: number | bigint): Promise<Uint8Array>;
  encrypt_uint256(v: number | bigint): Promise<Uint8Array>;
  encrypt_address(a: string | bigint): Promise<Uint8Array>;
  /** requests submitted concurrently share PBS launches (lockstep circuit levels) */
  evaluate(req: EvaluateRequest): Promise<Uint8Array>;
  decrypt(ct: Uint8Array): Promise<bigint>;
  decryptSync(ct: Uint8Array): bigint;
  unseal(address: string, sealedData: Uint8Array | string): bigint;
  close(): void;
}
