'use strict';
/**
 * Radix integers on P-FHEVM — the JS twin of tfhe_amd/radix.py (fhEVM's own representation:
 * w/2 blocks of 2-bit message + 2-bit carry, value v < 16 encoded v * 2^63/16 under the big key).
 * Operators are generator coroutines yielding one level of [lin (BigUint64Array of B blocks), table]
 * requests; RadixCircuit.runMany bootstraps each level of all operators in ONE multi-LUT PBS launch.
 * Semantics and circuits match radix.py exactly (same tables, same levels).
 */
const MSG = 4;
const SPACE = 16;
const DELTA = (1n << 63n) / 16n;

const table = (f) => Array.from({ length: SPACE }, (_, v) => ((Number(f(v)) % SPACE) + SPACE) % SPACE);
const biv = (f) => table((v) => f(Math.floor(v / MSG), v % MSG));

const T = {
  MSG: table((v) => v % MSG),
  STATE: table((v) => (v >= MSG ? 2 : v === MSG - 1 ? 1 : 0)),
  MERGE: biv((hi, lo) => (hi === 1 ? lo : hi)),
  APPLY: biv((st, m) => (m + (st === 2 ? 1 : 0)) % MSG),
  AND: biv((x, y) => x & y),
  OR: biv((x, y) => x | y),
  XOR: biv((x, y) => x ^ y),
  EQ: biv((x, y) => (x === y ? 1 : 0)),
  AND1: biv((x, y) => x & y & 1),
  CMP: biv((x, y) => (x < y ? 0 : x === y ? 1 : 2)),
  SEL_T: biv((c, x) => (c === 1 ? x : 0)),
  SEL_F: biv((c, x) => (c === 1 ? 0 : x)),
  MUL_LO: biv((x, y) => (x * y) % MSG),
  MUL_HI: biv((x, y) => Math.floor((x * y) / MSG)),
  CARRY: table((v) => Math.floor(v / MSG)),
  SHL_LO: biv((cur, prev) => ((cur << 1) | (prev >> 1)) & 3),
  SHR_LO: biv((nxt, cur) => ((cur >> 1) | (nxt << 1)) & 3),
  BIT0: table((v) => v & 1),
  BIT1: table((v) => (v >> 1) & 1),
};
const IS = { lt: table((v) => +(v === 0)), le: table((v) => +(v <= 1)), gt: table((v) => +(v === 2)), ge: table((v) => +(v >= 1)) };

class RadixCircuit {
  /** engine: { params: {k, N, n, order}, async pbs(cts, luts, lutIndex), lutFromTable(table) } */
  constructor(engine) {
    this.engine = engine;
    const p = engine.params;
    this.dim = p.order === 1 ? p.k * p.N + 1 : p.n + 1;
    this.luts = new Map();
    this.pbsCount = 0;
    this.launches = 0;
  }
  lut(tab) {
    const key = tab.join(',');
    if (!this.luts.has(key)) this.luts.set(key, this.engine.lutFromTable(tab));
    return this.luts.get(key);
  }
  /** B trivial blocks (columns) of clear values */
  trivial(vals) {
    const out = new BigUint64Array(vals.length * this.dim);
    vals.forEach((v, i) => { out[(i + 1) * this.dim - 1] = BigInt.asUintN(64, (BigInt(v) % 16n) * DELTA); });
    return out;
  }
  const(B, v) { return this.trivial(new Array(B).fill(v)); }
  add(...xs) {
    const out = xs[0].slice();
    for (let t = 1; t < xs.length; t++) { const x = xs[t]; for (let i = 0; i < out.length; i++) out[i] = BigInt.asUintN(64, out[i] + x[i]); }
    return out;
  }
  pack(x, y) {
    const out = new BigUint64Array(x.length);
    for (let i = 0; i < x.length; i++) out[i] = BigInt.asUintN(64, x[i] * 4n + y[i]);
    return out;
  }
  not(a) {
    const B = a.length / this.dim;
    const out = this.const(B, MSG - 1);
    for (let i = 0; i < out.length; i++) out[i] = BigInt.asUintN(64, out[i] - a[i]);
    return out;
  }
  async bootstrap(reqs) {
    if (!reqs.length) return [];
    const tabs = [];
    const index = new Map();
    let total = 0;
    for (const [lin] of reqs) total += lin.length;
    const flat = new BigUint64Array(total);
    const idx = new Uint32Array(total / this.dim);
    let off = 0;
    for (const [lin, tab] of reqs) {
      const key = tab.join(',');
      if (!index.has(key)) { index.set(key, tabs.length); tabs.push(tab); }
      flat.set(lin, off);
      idx.fill(index.get(key), off / this.dim, (off + lin.length) / this.dim);
      off += lin.length;
    }
    const N = this.engine.params.N;
    const luts = new BigUint64Array(tabs.length * N);
    tabs.forEach((t, i) => luts.set(this.lut(t), i * N));
    const out = await this.engine.pbs(flat, luts, idx);
    this.pbsCount += total / this.dim;
    this.launches += 1;
    const res = [];
    off = 0;
    for (const [lin] of reqs) { res.push(out.slice(off, off + lin.length)); off += lin.length; }
    return res;
  }
  async run(gen) { return (await this.runMany([gen]))[0]; }
  async runMany(gens) {
    const results = new Array(gens.length);
    const pending = new Map();
    gens.forEach((g, i) => { const r = g.next(); if (r.done) results[i] = r.value; else pending.set(i, { g, lvl: r.value }); });
    while (pending.size) {
      const order = Array.from(pending.keys());
      const reqs = [];
      const counts = [];
      for (const i of order) { reqs.push(...pending.get(i).lvl); counts.push(pending.get(i).lvl.length); }
      const outs = await this.bootstrap(reqs);
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
}

/** B values of width w: blocks[j] = column of block j (B ciphertexts), LSB block first */
class RadixVec {
  constructor(c, blocks, B) { this.c = c; this.blocks = blocks; this.B = B; }
  get width() { return 2 * this.blocks.length; }
  static digits(values, w) { return Array.from({ length: w / 2 }, (_, j) => values.map((v) => Number((BigInt(v) >> BigInt(2 * j)) & 3n))); }
  static trivial(c, values, w) { return new RadixVec(c, RadixVec.digits(values, w).map((d) => c.trivial(d)), values.length); }
  /** value-major [B][w/2][dim] <-> columns */
  static fromValueMajor(c, ct, B, nb) {
    const d = c.dim;
    const blocks = [];
    for (let j = 0; j < nb; j++) {
      const col = new BigUint64Array(B * d);
      for (let i = 0; i < B; i++) col.set(ct.subarray((i * nb + j) * d, (i * nb + j + 1) * d), i * d);
      blocks.push(col);
    }
    return new RadixVec(c, blocks, B);
  }
  toValueMajor() {
    const d = this.c.dim, nb = this.blocks.length, B = this.B;
    const out = new BigUint64Array(B * nb * d);
    for (let j = 0; j < nb; j++) for (let i = 0; i < B; i++) out.set(this.blocks[j].subarray(i * d, (i + 1) * d), (i * nb + j) * d);
    return out;
  }
  cast(w) {
    const nb = w / 2;
    if (nb === this.blocks.length) return this;
    if (nb < this.blocks.length) return new RadixVec(this.c, this.blocks.slice(0, nb), this.B);
    const pad = Array.from({ length: nb - this.blocks.length }, () => this.c.const(this.B, 0));
    return new RadixVec(this.c, this.blocks.concat(pad), this.B);
  }
}

function* gPropagate(c, s, B, carryIn) {
  const nb = s.length;
  if (carryIn) s = [c.add(s[0], c.const(B, 1))].concat(s.slice(1));
  const o = yield s.map((x) => [x, T.MSG]).concat(s.map((x) => [x, T.STATE]));
  const msg = o.slice(0, nb);
  let st = o.slice(nb);
  for (let d = 1; d < nb; d *= 2) {
    const merged = yield st.slice(d).map((hi, i) => [c.pack(hi, st[i]), T.MERGE]);
    st = st.slice(0, d).concat(merged);
  }
  if (nb === 1) return msg;
  const hi = yield msg.slice(1).map((m, i) => [c.pack(st[i], m), T.APPLY]);
  return [msg[0]].concat(hi);
}

function* gSumColumns(c, cols, B) {
  const nb = cols.length;
  while (Math.max(...cols.map((col) => col.length)) > 2) {
    const reqs = [];
    const plan = [];
    const next = Array.from({ length: nb }, () => []);
    cols.forEach((col, k) => {
      if (col.length <= 2) { next[k].push(...col); return; }
      for (let g = 0; g < col.length; g += 5) {
        const grp = col.slice(g, g + 5);
        if (grp.length === 1) { next[k].push(grp[0]); continue; }
        const ssum = c.add(...grp);
        reqs.push([ssum, T.MSG], [ssum, T.CARRY]);
        plan.push(k);
      }
    });
    const outs = yield reqs;
    plan.forEach((k, t) => { next[k].push(outs[2 * t]); if (k + 1 < nb) next[k + 1].push(outs[2 * t + 1]); });
    cols = next;
  }
  const zero = () => c.const(B, 0);
  const a = cols.map((col) => (col.length > 0 ? col[0] : zero()));
  const b = cols.map((col) => (col.length > 1 ? col[1] : zero()));
  return yield* gPropagate(c, a.map((x, i) => c.add(x, b[i])), B, false);
}

function* gMul(c, a, b, B) {
  const nb = a.length;
  const reqs = [];
  const pos = [];
  if (typeof b === 'bigint') {
    const digs = Array.from({ length: nb }, (_, j) => Number((b >> BigInt(2 * j)) & 3n));
    for (let i = 0; i < nb; i++) {
      for (let j = 0; j < nb - i; j++) {
        const d = digs[j];
        if (!d) continue;
        reqs.push([a[i], table((v) => (v * d) % MSG)]); pos.push(i + j);
        if (i + j + 1 < nb) { reqs.push([a[i], table((v) => Math.floor((v * d) / MSG))]); pos.push(i + j + 1); }
      }
    }
  } else {
    for (let i = 0; i < nb; i++) {
      for (let j = 0; j < nb - i; j++) {
        const pk = c.pack(a[i], b[j]);
        reqs.push([pk, T.MUL_LO]); pos.push(i + j);
        if (i + j + 1 < nb) { reqs.push([pk, T.MUL_HI]); pos.push(i + j + 1); }
      }
    }
  }
  const cols = Array.from({ length: nb }, () => []);
  if (reqs.length) { const outs = yield reqs; outs.forEach((o, t) => cols[pos[t]].push(o)); }
  return yield* gSumColumns(c, cols, B);
}

function* gEq(c, a, b, B) {
  let e = yield a.map((x, i) => [c.pack(x, b[i]), T.EQ]);
  while (e.length > 1) {
    if (e.length % 2) e = e.concat([c.const(B, 1)]);
    const lvl = [];
    for (let k = 0; k < e.length; k += 2) lvl.push([c.pack(e[k], e[k + 1]), T.AND1]);
    e = yield lvl;
  }
  return e[0];
}

function* gCmp(c, a, b, B) {
  let st = yield a.map((x, i) => [c.pack(x, b[i]), T.CMP]);
  while (st.length > 1) {
    if (st.length % 2) st = st.concat([c.const(B, 1)]);
    const lvl = [];
    for (let k = 0; k < st.length; k += 2) lvl.push([c.pack(st[k + 1], st[k]), T.MERGE]);
    st = yield lvl;
  }
  return st[0];
}

function* gSelect(c, cond, x, y) {
  const tf = yield x.map((xi) => [c.pack(cond, xi), T.SEL_T]).concat(y.map((yi) => [c.pack(cond, yi), T.SEL_F]));
  const n = x.length;
  return yield tf.slice(0, n).map((t, i) => [c.add(t, tf[n + i]), T.MSG]);
}

function* gShift(c, a, k, kind, B) {
  const nb = a.length;
  const w = 2 * nb;
  k %= w;
  const q = Math.floor(k / 2), r = k % 2;
  const zero = () => c.const(B, 0);
  const rot = kind === 'rotl' || kind === 'rotr';
  const roll = (arr, sh) => { const n = arr.length; sh = ((sh % n) + n) % n; return arr.slice(n - sh).concat(arr.slice(0, n - sh)); };
  if (kind === 'shl' || kind === 'rotl') {
    const moved = rot ? roll(a, q) : Array.from({ length: q }, zero).concat(a.slice(0, nb - q));
    if (!r) return moved;
    const prev = rot ? roll(moved, 1) : [zero()].concat(moved.slice(0, -1));
    return yield moved.map((m, i) => [c.pack(m, prev[i]), T.SHL_LO]);
  }
  const moved = rot ? roll(a, -q) : a.slice(q).concat(Array.from({ length: q }, zero));
  if (!r) return moved;
  const nxt = rot ? roll(moved, -1) : moved.slice(1).concat([zero()]);
  return yield moved.map((m, i) => [c.pack(nxt[i], m), T.SHR_LO]);
}

function* gShiftEnc(c, a, amount, kind, B) {
  const w = 2 * a.length;
  const nbits = Math.max(1, (w - 1).toString(2).length);
  const bits = yield Array.from({ length: nbits }, (_, k) => [amount[k >> 1], k % 2 ? T.BIT1 : T.BIT0]);
  let cur = a;
  for (let k = 0; k < nbits; k++) {
    const moved = yield* gShift(c, cur, 1 << k, kind, B);
    cur = yield* gSelect(c, bits[k], moved, cur);
  }
  return cur;
}

const T_LOW_BIT = table((v) => v & 1);

/** (a / d, a % d) for a plaintext divisor by multiply-high (radix.py g_div_rem_scalar) */
function* gDivRemScalar(c, a, d, B) {
  const nb = a.length;
  const w = 2 * nb;
  d = BigInt.asUintN(w, BigInt(d));
  if (d === 0n) return [a.map(() => c.const(B, MSG - 1)), a];
  if ((d & (d - 1n)) === 0n) {
    const s = d.toString(2).length - 1;
    const q = s ? yield* gShift(c, a, s, 'shr', B) : a;
    const keep = Math.floor(s / 2);
    const rem = a.slice(0, keep);
    if (s % 2) rem.push((yield [[a[keep], T_LOW_BIT]])[0]);
    while (rem.length < nb) rem.push(c.const(B, 0));
    return [q, rem];
  }
  const l = BigInt((d - 1n).toString(2).length);
  const W = BigInt(w);
  const m = ((1n << (W + l)) + d - 1n) / d;
  const nbw = w + 1;
  const aExt = a.concat(Array.from({ length: nbw - nb }, () => c.const(B, 0)));
  const prod = yield* gMul(c, aExt, m, B);
  const k = w + Number(l);
  let sub = prod.slice(Math.floor(k / 2), Math.floor(k / 2) + nb + 1);
  while (sub.length < nb + 1) sub.push(c.const(B, 0));
  const q = (k % 2 ? yield* gShift(c, sub, 1, 'shr', B) : sub).slice(0, nb);
  const qd = yield* gMul(c, q, d, B);
  const r = yield* gPropagate(c, a.map((x, i) => c.add(x, c.not(qd[i]))), B, true);
  return [q, r];
}

const RADIX_OPS = ['add', 'sub', 'mul', 'div', 'rem', 'and', 'or', 'xor', 'eq', 'ne', 'lt', 'le', 'gt', 'ge', 'min', 'max', 'neg', 'not', 'shl', 'shr', 'rotl', 'rotr'];

/** one fhEVM operator on radix values (lhs/rhs: RadixVec or plaintext bigint); bool results are a block column */
function* fhevmOp(c, op, lhs, rhs = null) {
  if (!RADIX_OPS.includes(op)) throw new Error(`radix operator ${op} not supported`);
  const isV = (x) => x instanceof RadixVec;
  if (op === 'not') return new RadixVec(c, lhs.blocks.map((b) => c.not(b)), lhs.B);
  if (op === 'neg') {
    const z = lhs.blocks.map(() => c.const(lhs.B, 0));
    return new RadixVec(c, yield* gPropagate(c, z.map((x, i) => c.add(x, c.not(lhs.blocks[i]))), lhs.B, true), lhs.B);
  }
  const lE = isV(lhs), rE = isV(rhs);
  if (!lE && !rE) throw new Error('at least one operand must be encrypted');
  if (['shl', 'shr', 'rotl', 'rotr'].includes(op)) {
    if (!lE) throw new Error('shift of a plaintext by an encrypted amount is not an fhEVM overload');
    if (rE) return new RadixVec(c, yield* gShiftEnc(c, lhs.blocks, rhs.blocks, op, lhs.B), lhs.B);
    return new RadixVec(c, yield* gShift(c, lhs.blocks, Number(BigInt(rhs) % BigInt(lhs.width)), op, lhs.B), lhs.B);
  }
  if (op === 'div' || op === 'rem') {
    if (!lE || rE) throw new Error('fhEVM div / rem take an encrypted numerator and a plaintext divisor');
    const [q, r] = yield* gDivRemScalar(c, lhs.blocks, rhs, lhs.B);
    return new RadixVec(c, op === 'div' ? q : r, lhs.B);
  }
  const w = Math.max(...[lhs, rhs].filter(isV).map((x) => x.width));
  const B = (lE ? lhs : rhs).B;
  const blocks = (x) => (isV(x) ? x.cast(w).blocks
    : RadixVec.digits(new Array(B).fill(BigInt.asUintN(w, BigInt(x))), w).map((d) => c.trivial(d)));
  if (op === 'mul') {
    if (!lE) return new RadixVec(c, yield* gMul(c, rhs.cast(w).blocks, BigInt.asUintN(w, BigInt(lhs)), B), B);
    if (!rE) return new RadixVec(c, yield* gMul(c, lhs.cast(w).blocks, BigInt.asUintN(w, BigInt(rhs)), B), B);
    return new RadixVec(c, yield* gMul(c, blocks(lhs), blocks(rhs), B), B);
  }
  const a = blocks(lhs), b = blocks(rhs);
  if (op === 'add') return new RadixVec(c, yield* gPropagate(c, a.map((x, i) => c.add(x, b[i])), B, false), B);
  if (op === 'sub') return new RadixVec(c, yield* gPropagate(c, a.map((x, i) => c.add(x, c.not(b[i]))), B, true), B);
  if (op === 'and' || op === 'or' || op === 'xor') {
    const t = { and: T.AND, or: T.OR, xor: T.XOR }[op];
    return new RadixVec(c, yield a.map((x, i) => [c.pack(x, b[i]), t]), B);
  }
  if (op === 'eq' || op === 'ne') {
    const e = yield* gEq(c, a, b, B);
    if (op === 'eq') return e;
    const one = c.const(B, 1);
    for (let i = 0; i < one.length; i++) one[i] = BigInt.asUintN(64, one[i] - e[i]);
    return one;
  }
  const st = yield* gCmp(c, a, b, B);
  if (op in IS) return (yield [[st, IS[op]]])[0];
  const takeA = (yield [[st, op === 'min' ? IS.lt : IS.gt]])[0];
  return new RadixVec(c, yield* gSelect(c, takeA, a, b), B);
}

/** decrypt a radix value batch with a ClientKey (shortint decoding mod 16 per block) */
function decryptRadix(clientKey, vec) {
  const vals = new Array(vec.B).fill(0n);
  vec.blocks.forEach((col, j) => {
    const d = clientKey.decrypt(col, SPACE);
    for (let i = 0; i < vec.B; i++) vals[i] += BigInt(d[i]) << BigInt(2 * j);
  });
  const m = (1n << BigInt(vec.width)) - 1n;
  return vals.map((v) => v & m);
}

module.exports = { MSG, SPACE, DELTA, T, RadixCircuit, RadixVec, fhevmOp, decryptRadix, RADIX_OPS };
