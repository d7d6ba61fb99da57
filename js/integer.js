'use strict';
/**
 * Encrypted unsigned integers on the GPU gate bootstrap — the JS twin of tfhe_amd/integer.py
 * (SURVEY §8f f1).  An encrypted w-bit integer batch is w "columns" (LSB first); column i is a
 * BigUint64Array holding bit i of all B values as B consecutive LWE ciphertexts (n + 1 words).
 *
 * Operators are generator coroutines that yield one circuit LEVEL (an array of columns of linear
 * combinations) and receive the bootstrapped columns; Circuit.runMany steps independent operators
 * in lockstep so each level of all of them is ONE engine.pbs launch.  Gates (inputs +-1/8):
 *   AND = PBS(a+b-1/8)  OR = PBS(a+b+1/8)  XOR = PBS(2(a+b)+1/4)  MAJ = PBS(a+b+c)
 *   XOR3 = PBS(-2(a+b+c))  NOT = -a (free)
 * Semantics are the fhEVM operators of the reference's KATs
 * (tests/fhevm-suite/e2e/test/fhevmOperations*.ts): wrapping add/sub/mul, neg, bitwise, comparisons
 * to ebool, min/max, shifts/rotations by amount mod w, div/rem by a plaintext, mixed widths
 * zero-extended to the wider type.
 */
const MU = 1n << 61n;

function lin(terms, c, dim) {
  const n = terms[0][1].length;
  const out = new BigUint64Array(n);
  for (let i = 0; i < n; i++) {
    let v = 0n;
    for (let t = 0; t < terms.length; t++) v += terms[t][1][i] * terms[t][0];
    out[i] = BigInt.asUintN(64, v);
  }
  if (c) for (let i = dim - 1; i < n; i += dim) out[i] = BigInt.asUintN(64, out[i] + c);
  return out;
}

class Circuit {
  /** engine: { params: {n}, gateLut(), async pbs(cts: BigUint64Array, lut) } */
  constructor(engine, capacity = 2048, roundSize = 1024) {
    this.engine = engine;
    this.dim = engine.params.n + 1;
    this.lut = engine.gateLut();
    this.capacity = capacity;
    this.roundSize = roundSize;  // PBS per batch-kernel round: the carry-out circuit's cost model
    this.pbsCount = 0;
    this.launches = 0;
  }
  AND(a, b) { return lin([[1n, a], [1n, b]], -MU, this.dim); }
  OR(a, b) { return lin([[1n, a], [1n, b]], MU, this.dim); }
  XOR(a, b) { return lin([[2n, a], [2n, b]], 2n * MU, this.dim); }
  MAJ(a, b, c) { return lin([[1n, a], [1n, b], [1n, c]], 0n, this.dim); }
  XOR3(a, b, c) { return lin([[-2n, a], [-2n, b], [-2n, c]], 0n, this.dim); }
  NOT(a) { return lin([[-1n, a]], 0n, this.dim); }

  /** noise-free encryptions (0, ..., 0, +-1/8) of clear bits */
  trivial(bits) {
    const out = new BigUint64Array(bits.length * this.dim);
    for (let i = 0; i < bits.length; i++) out[(i + 1) * this.dim - 1] = bits[i] ? MU : BigInt.asUintN(64, -MU);
    return out;
  }
  trivialConst(bit, B) { return this.trivial(new Array(B).fill(!!bit)); }

  async bootstrap(cols) {
    const total = cols.reduce((s, c) => s + c.length, 0);
    if (total === 0) return cols.map((c) => c.slice());
    const flat = new BigUint64Array(total);
    let off = 0;
    for (const c of cols) { flat.set(c, off); off += c.length; }
    const out = await this.engine.pbs(flat, this.lut);
    this.pbsCount += total / this.dim;
    this.launches += 1;
    const res = [];
    off = 0;
    for (const c of cols) { res.push(out.slice(off, off + c.length)); off += c.length; }
    return res;
  }

  async run(gen) { return (await this.runMany([gen]))[0]; }

  async runMany(gens) {
    const results = new Array(gens.length);
    const pending = new Map();
    gens.forEach((g, i) => {
      const r = g.next();
      if (r.done) results[i] = r.value; else pending.set(i, { g, lvl: r.value });
    });
    while (pending.size) {
      const order = Array.from(pending.keys());
      const cols = [];
      const counts = [];
      for (const i of order) { cols.push(...pending.get(i).lvl); counts.push(pending.get(i).lvl.length); }
      const outs = await this.bootstrap(cols);
      let off = 0;
      order.forEach((i, k) => {
        const { g } = pending.get(i);
        const r = g.next(outs.slice(off, off + counts[k]));
        off += counts[k];
        if (r.done) { results[i] = r.value; pending.delete(i); } else pending.set(i, { g, lvl: r.value });
      });
    }
    return results;
  }

  preferPrefix(B, w) { return B * w * 2 <= this.capacity; }

  /** block size of carryOut with the fewest launch rounds, then the fewest PBS (tfhe_amd/integer.py twin) */
  carryBlock(B, w) {
    const cands = new Set([w]);
    for (let s = 1; s <= w; s *= 2) cands.add(s);
    let best = null;
    for (const s of [...cands].sort((x, y) => x - y)) {
      const lv = carryLevels(B, w, s);
      const key = [lv.reduce((t, n) => t + Math.max(1, Math.ceil(n / this.roundSize)), 0), lv.reduce((t, n) => t + n, 0), -s];
      if (best === null || key[0] < best[0][0] || (key[0] === best[0][0] && (key[1] < best[0][1] ||
          (key[1] === best[0][1] && key[2] < best[0][2])))) best = [key, s];
    }
    return best[1];
  }
}

/** PBS per launch of carryOut(width w, block size s) over a batch of B */
function carryLevels(B, w, s) {
  const nb = Math.ceil(w / s);
  const lv = [];
  for (let j = 0; j < s; j++) {
    let act = 0;
    for (let k = 1; k < nb; k++) if (k * s + j < w) act++;
    lv.push(B * (1 + 2 * act));
  }
  for (let n = nb; n > 1; n -= Math.floor(n / 2)) lv.push(B * (1 + 2 * (Math.floor(n / 2) - 1)));
  return lv;
}

/** an encrypted batch: B values of width w, columns LSB first */
class FheUintVec {
  constructor(circuit, cols, B) { this.c = circuit; this.cols = cols; this.B = B; }
  get width() { return this.cols.length; }
  static bitsOf(values, w) {
    return Array.from({ length: w }, (_, j) => values.map((v) => ((BigInt(v) >> BigInt(j)) & 1n) === 1n));
  }
  static trivial(circuit, values, w) {
    return new FheUintVec(circuit, FheUintVec.bitsOf(values, w).map((b) => circuit.trivial(b)), values.length);
  }
  /** clientKey.encryptBool(bits, seed, stream0) -> BigUint64Array; bit j of value i uses stream stream0 + i*w + j */
  static encrypt(circuit, clientKey, values, w, seed = 1n, stream0 = 0n) {
    const B = values.length;
    const flat = [];
    for (const v of values) for (let j = 0; j < w; j++) flat.push(((BigInt(v) >> BigInt(j)) & 1n) === 1n);
    const ct = clientKey.encryptBool(flat, seed, stream0);
    return FheUintVec.fromValueMajor(circuit, ct, B, w);
  }
  /** value-major layout [B][w][dim] (the serialized / C-ABI layout) -> columns */
  static fromValueMajor(circuit, ct, B, w) {
    const d = circuit.dim;
    const cols = [];
    for (let j = 0; j < w; j++) {
      const col = new BigUint64Array(B * d);
      for (let i = 0; i < B; i++) col.set(ct.subarray((i * w + j) * d, (i * w + j + 1) * d), i * d);
      cols.push(col);
    }
    return new FheUintVec(circuit, cols, B);
  }
  toValueMajor() {
    const d = this.c.dim, w = this.width, B = this.B;
    const out = new BigUint64Array(B * w * d);
    for (let j = 0; j < w; j++) for (let i = 0; i < B; i++) out.set(this.cols[j].subarray(i * d, (i + 1) * d), (i * w + j) * d);
    return out;
  }
  decrypt(clientKey) { return decryptColumns(clientKey, this.cols, this.B); }
  cast(w) {
    if (w === this.width) return this;
    if (w < this.width) return new FheUintVec(this.c, this.cols.slice(0, w), this.B);
    const pad = Array.from({ length: w - this.width }, () => this.c.trivialConst(false, this.B));
    return new FheUintVec(this.c, this.cols.concat(pad), this.B);
  }
}

function decryptColumns(clientKey, cols, B) {
  const vals = new Array(B).fill(0n);
  cols.forEach((col, j) => {
    const bits = clientKey.decryptBool(col);
    for (let i = 0; i < B; i++) if (bits[i]) vals[i] |= 1n << BigInt(j);
  });
  return vals;
}

// ------------------------------------------------------------------------------------------
// circuits (columns in, columns out)
// ------------------------------------------------------------------------------------------
function* gBitwise(c, kind, a, b) {
  const gate = { and: (x, y) => c.AND(x, y), or: (x, y) => c.OR(x, y), xor: (x, y) => c.XOR(x, y) }[kind];
  return yield a.map((x, i) => gate(x, b[i]));
}

/** carry-out of a + b + cin in blocks of s bits: block ripple in lockstep (block 0 from the known carry-in,
 * blocks k >= 1 for both carry-ins G / P), then a reduction tree of (G, P) merges onto block 0 */
function* carryOut(c, a, b, B, cin, s) {
  const w = a.length, nb = Math.ceil(w / s);
  let C = c.trivialConst(cin, B);
  let G = [], P = [];
  for (let j = 0; j < s; j++) {
    const ks = [];
    for (let k = 1; k < nb; k++) if (k * s + j < w) ks.push(k);
    const m = ks.length;
    const lvl = [c.MAJ(a[j], b[j], C)];
    if (j === 0) {
      for (const k of ks) lvl.push(c.AND(a[k * s], b[k * s]));
      for (const k of ks) lvl.push(c.OR(a[k * s], b[k * s]));
    } else {
      ks.forEach((k, i) => lvl.push(c.MAJ(a[k * s + j], b[k * s + j], G[i])));
      ks.forEach((k, i) => lvl.push(c.MAJ(a[k * s + j], b[k * s + j], P[i])));
    }
    const out = yield lvl;
    C = out[0];
    G = out.slice(1, 1 + m).concat(G.slice(m));
    P = out.slice(1 + m, 1 + 2 * m).concat(P.slice(m));
  }
  while (G.length > 0) {
    const n = G.length + 1, np = Math.floor(n / 2) - 1;
    const lvl = [c.MAJ(G[0], P[0], C)];
    for (let i = 1; i <= np; i++) lvl.push(c.MAJ(G[2 * i], P[2 * i], G[2 * i - 1]));
    for (let i = 1; i <= np; i++) lvl.push(c.MAJ(G[2 * i], P[2 * i], P[2 * i - 1]));
    const out = yield lvl;
    C = out[0];
    const nG = out.slice(1, 1 + np), nP = out.slice(1 + np, 1 + 2 * np);
    if (n % 2) { nG.push(G[n - 2]); nP.push(P[n - 2]); }
    G = nG; P = nP;
  }
  return C;
}

function* gAdd(c, a, b, B, cin = false, wantSum = true, wantCarry = false, prefix = null) {
  const w = a.length;
  if (!wantSum) {
    const s = prefix === null ? c.carryBlock(B, w) : (prefix ? 1 : w);
    return [null, yield* carryOut(c, a, b, B, cin, s)];
  }
  if (prefix === null) prefix = c.preferPrefix(B, w);
  if (!prefix) {
    let carry = c.trivialConst(cin, B);
    const sums = [];
    for (let i = 0; i < w; i++) {
      const lvl = [];
      const needCarry = i < w - 1 || wantCarry;
      if (needCarry) lvl.push(c.MAJ(a[i], b[i], carry));
      if (wantSum) lvl.push(c.XOR3(a[i], b[i], carry));
      const out = yield lvl;
      if (wantSum) sums.push(out[out.length - 1]);
      if (needCarry) carry = out[0];
    }
    return [wantSum ? sums : null, wantCarry ? carry : null];
  }
  const gp = yield a.map((x, i) => c.AND(x, b[i])).concat(a.map((x, i) => c.OR(x, b[i])));
  let G = gp.slice(0, w), P = gp.slice(w);
  for (let d = 1; d < w; d *= 2) {
    const lvl = [];
    for (let i = d; i < w; i++) lvl.push(c.MAJ(G[i], P[i], G[i - d]));
    for (let i = d; i < w; i++) lvl.push(c.MAJ(G[i], P[i], P[i - d]));
    const out = yield lvl;
    const m = w - d;
    G = G.slice(0, d).concat(out.slice(0, m));
    P = P.slice(0, d).concat(out.slice(m));
  }
  const pref = cin ? P : G;
  const carries = [c.trivialConst(cin, B)].concat(pref.slice(0, w - 1));
  const s = yield a.map((x, i) => c.XOR3(x, b[i], carries[i]));
  return [s, wantCarry ? pref[w - 1] : null];
}

function* gGe(c, a, b, B) {
  const r = yield* gAdd(c, a, b.map((x) => c.NOT(x)), B, true, false, true);
  return r[1];
}

function* gEq(c, a, b, B) {
  let cur = (yield a.map((x, i) => c.XOR(x, b[i]))).map((x) => c.NOT(x));
  while (cur.length > 1) {
    if (cur.length % 2) cur = cur.concat([c.trivialConst(true, B)]);
    const lvl = [];
    for (let k = 0; k < cur.length; k += 2) lvl.push(c.AND(cur[k], cur[k + 1]));
    cur = yield lvl;
  }
  return cur[0];
}

function* gSelect(c, cond, x, y) {
  const ncond = c.NOT(cond);
  const tf = yield x.map((xi) => c.AND(cond, xi)).concat(y.map((yi) => c.AND(ncond, yi)));
  const w = x.length;
  // at most one of t, f is true: OR(t, f) = t + f + 1/8 exactly, no second bootstrap (tfhe_amd/integer.py)
  return tf.slice(0, w).map((t, i) => c.OR(t, tf[w + i]));
}

function* gMul(c, a, b, B) {
  const w = a.length;
  const zero = () => c.trivialConst(false, B);
  let rows = [];
  if (typeof b === 'bigint') {
    const k = BigInt.asUintN(w, b);
    for (let j = 0; j < w; j++) {
      if ((k >> BigInt(j)) & 1n) rows.push(Array.from({ length: j }, zero).concat(a.slice(0, w - j)));
    }
  } else {
    const lvl = [];
    const idx = [];
    for (let j = 0; j < w; j++) for (let i = 0; i < w - j; i++) { lvl.push(c.AND(a[i], b[j])); idx.push(j); }
    const pp = yield lvl;
    let off = 0;
    for (let j = 0; j < w; j++) {
      rows.push(Array.from({ length: j }, zero).concat(pp.slice(off, off + w - j)));
      off += w - j;
    }
  }
  if (!rows.length) return Array.from({ length: w }, zero);
  while (rows.length > 2) {
    const nt = Math.floor(rows.length / 3);
    const lvl = [];
    for (let t = 0; t < nt; t++) {
      const [x, y, z] = rows.slice(3 * t, 3 * t + 3);
      for (let i = 0; i < w; i++) lvl.push(c.XOR3(x[i], y[i], z[i]));
      for (let i = 0; i < w - 1; i++) lvl.push(c.MAJ(x[i], y[i], z[i]));
    }
    const out = yield lvl;
    const nrows = [];
    for (let t = 0; t < nt; t++) {
      const base = t * (2 * w - 1);
      nrows.push(out.slice(base, base + w));
      nrows.push([zero()].concat(out.slice(base + w, base + 2 * w - 1)));
    }
    rows = nrows.concat(rows.slice(3 * nt));
  }
  if (rows.length === 1) return rows[0];
  return (yield* gAdd(c, rows[0], rows[1], B))[0];
}

function* gDivRemScalar(c, a, d, B) {
  const w = a.length;
  d = BigInt.asUintN(w, BigInt(d));
  if (d === 0n) return [Array.from({ length: w }, () => c.trivialConst(true, B)), a];
  const L = d.toString(2).length;
  const q = Array.from({ length: w }, () => c.trivialConst(false, B));
  let R = a.slice(w - (L - 1));
  for (let i = w - L; i >= 0; i--) {
    R = [a[i]].concat(R);
    const r = R.length;
    const nd = Array.from({ length: r }, (_, j) => c.trivialConst(((d >> BigInt(j)) & 1n) === 0n, B));
    const [t, ge] = yield* gAdd(c, R, nd, B, true, true, true);
    q[i] = ge;
    R = yield* gSelect(c, ge, t, R);
    if (r > L) R = R.slice(0, L);
  }
  const rem = R.length < w ? R.concat(Array.from({ length: w - R.length }, () => c.trivialConst(false, B))) : R.slice(0, w);
  return [q, rem];
}

function shiftClear(c, a, k, kind, B) {
  const w = a.length;
  k %= w;
  const zeros = Array.from({ length: k }, () => c.trivialConst(false, B));
  if (kind === 'shl') return zeros.concat(a.slice(0, w - k));
  if (kind === 'shr') return a.slice(k).concat(zeros);
  if (kind === 'rotl') return a.slice(w - k).concat(a.slice(0, w - k));
  if (kind === 'rotr') return a.slice(k).concat(a.slice(0, k));
  throw new Error(`unknown shift ${kind}`);
}

function* gShift(c, a, amount, kind, B) {
  if (typeof amount === 'number') return shiftClear(c, a, amount, kind, B);
  const w = a.length;
  let cur = a;
  const nb = Math.max(1, (w - 1).toString(2).length);
  for (let k = 0; k < nb; k++) cur = yield* gSelect(c, amount[k], shiftClear(c, cur, 1 << k, kind, B), cur);
  return cur;
}

const BINARY_OPS = ['add', 'sub', 'mul', 'div', 'rem', 'and', 'or', 'xor', 'shl', 'shr', 'rotl', 'rotr',
  'eq', 'ne', 'ge', 'gt', 'le', 'lt', 'min', 'max'];
const UNARY_OPS = ['neg', 'not'];
const BOOL_RESULT = ['eq', 'ne', 'ge', 'gt', 'le', 'lt'];

/**
 * One fhEVM operator as a coroutine.  lhs / rhs: FheUintVec or plaintext (number | bigint; at most
 * one plaintext).  Returns an FheUintVec, or for comparisons an encrypted-bool column.
 */
function* fhevmOp(c, op, lhs, rhs = null) {
  const isEnc = (x) => x instanceof FheUintVec;
  if (UNARY_OPS.includes(op)) {
    if (op === 'not') return new FheUintVec(c, lhs.cols.map((x) => c.NOT(x)), lhs.B);
    const zero = Array.from({ length: lhs.width }, () => c.trivialConst(false, lhs.B));
    const [s] = yield* gAdd(c, zero, lhs.cols.map((x) => c.NOT(x)), lhs.B, true);
    return new FheUintVec(c, s, lhs.B);
  }
  if (!BINARY_OPS.includes(op)) throw new Error(`unknown operator ${op}`);
  const lEnc = isEnc(lhs), rEnc = isEnc(rhs);
  if (!lEnc && !rEnc) throw new Error('at least one operand must be encrypted');
  if (['shl', 'shr', 'rotl', 'rotr'].includes(op)) {
    if (!lEnc) throw new Error('shift of a plaintext by an encrypted amount is not an fhEVM overload');
    let amt;
    if (rEnc) {
      const nb = Math.max(1, (lhs.width - 1).toString(2).length);
      amt = (rhs.width >= nb ? rhs : rhs.cast(nb)).cols;
    } else amt = Number(BigInt(rhs) % BigInt(lhs.width));
    return new FheUintVec(c, yield* gShift(c, lhs.cols, amt, op, lhs.B), lhs.B);
  }
  if (op === 'div' || op === 'rem') {
    if (!lEnc || rEnc) throw new Error('div/rem take an encrypted numerator and a plaintext divisor');
    const [q, r] = yield* gDivRemScalar(c, lhs.cols, BigInt(rhs), lhs.B);
    return new FheUintVec(c, op === 'div' ? q : r, lhs.B);
  }
  const w = Math.max(...[lhs, rhs].filter(isEnc).map((x) => x.width));
  const B = (lEnc ? lhs : rhs).B;
  const bits = (x) => (isEnc(x) ? x.cast(w).cols
    : FheUintVec.bitsOf(new Array(B).fill(BigInt.asUintN(w, BigInt(x))), w).map((col) => c.trivial(col)));
  if (op === 'mul') {
    if (!lEnc) return new FheUintVec(c, yield* gMul(c, rhs.cast(w).cols, BigInt(lhs), B), B);
    if (!rEnc) return new FheUintVec(c, yield* gMul(c, lhs.cast(w).cols, BigInt(rhs), B), B);
    return new FheUintVec(c, yield* gMul(c, bits(lhs), bits(rhs), B), B);
  }
  const a = bits(lhs), b = bits(rhs);
  if (op === 'and' || op === 'or' || op === 'xor') return new FheUintVec(c, yield* gBitwise(c, op, a, b), B);
  if (op === 'add') return new FheUintVec(c, (yield* gAdd(c, a, b, B))[0], B);
  if (op === 'sub') return new FheUintVec(c, (yield* gAdd(c, a, b.map((x) => c.NOT(x)), B, true))[0], B);
  if (op === 'eq' || op === 'ne') { const e = yield* gEq(c, a, b, B); return op === 'eq' ? e : c.NOT(e); }
  if (op === 'ge' || op === 'lt') { const g = yield* gGe(c, a, b, B); return op === 'ge' ? g : c.NOT(g); }
  if (op === 'le' || op === 'gt') { const g = yield* gGe(c, b, a, B); return op === 'le' ? g : c.NOT(g); }
  const lt = c.NOT(yield* gGe(c, a, b, B));
  if (op === 'min') return new FheUintVec(c, yield* gSelect(c, lt, a, b), B);
  return new FheUintVec(c, yield* gSelect(c, lt, b, a), B);
}

module.exports = { MU, Circuit, FheUintVec, fhevmOp, decryptColumns, BINARY_OPS, UNARY_OPS, BOOL_RESULT };
