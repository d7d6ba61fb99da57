"""Radix integers on the production fhEVM parameters (the representation tfhe-rs /
fhEVM use: PARAM_MESSAGE_2_CARRY_2_KS_PBS, sdk/relayer/src/tfhe.ts:14-19).

A w-bit encrypted integer is w/2 blocks (LSB first); each block is a big LWE (dim 2048) of a value
v in [0, 16) = 2-bit message + 2-bit carry space, encoded v * 2^63 / 16 (one padding bit).  A
"clean" block holds v < 4.  Every programmable bootstrap evaluates a 16-entry table on one block;
two clean blocks x, y combine into one PBS input 4x + y ("bivariate" LUT, tfhe-rs
`apply_bivariate_lookup_table`).  All PBS of one circuit level — across every value, block and
independent operation — run as ONE `Engine.pbs` launch with a per-ciphertext LUT index.

Operators (fhEVM semantics, as tfhe_amd.integer): add/sub/neg with parallel-prefix carry
propagation over block states {0: none, 1: propagate, 2: generate} (log2(blocks) levels),
bitwise and/or/xor (1 level), not (free: 3 - v), eq/ne (per-block equality + AND tree),
lt/le/gt/ge (per-block {<, =, >} + MSB-first merge tree), min/max (compare + 2-PBS select),
shl/shr/rotl/rotr by a plaintext amount (block moves + one bivariate level for odd shifts) or an
encrypted one (barrel shifter over the amount's bits), mul (block products by bivariate low/high
digit tables, carry-save reduction rounds of up to 5 blocks, final prefix add; plaintext factors by
univariate tables), div/rem by a plaintext divisor (multiply-high by a (w+1)-bit reciprocal),
plaintext right operands, mixed widths zero-extended.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

MSG = 4                     # message modulus
SPACE = 16                  # message x carry
DELTA = (1 << 63) // SPACE  # one padding bit
_M64 = 1 << 64


def _table(f: Callable[[int], int]) -> Tuple[int, ...]:
    return tuple(int(f(v)) % SPACE for v in range(SPACE))


def _biv(f: Callable[[int, int], int]) -> Tuple[int, ...]:
    """bivariate table on 4x + y (x, y < 4)."""
    return _table(lambda v: f(v // MSG, v % MSG))


MAX_LAUNCH = 1 << 18  # ciphertexts per engine call (P-FHEVM: 2 x 2049 x 8 B x 256 Ki = 8.6 GB of I/O)


class RadixCircuit:
    """Lockstep executor: each level is a list of (lin array (..., dim+1), table) pairs; every
    distinct table becomes one LUT of the launch and each ciphertext indexes its own."""

    def __init__(self, engine):
        self.engine = engine
        p = engine.params
        self.dim = p.k * p.N + 1 if p.order == 1 else p.n + 1
        self.N = p.N
        self._luts: Dict[Tuple[int, ...], np.ndarray] = {}
        self.pbs_count = 0
        self.launches = 0

    def lut(self, table: Tuple[int, ...]) -> np.ndarray:
        if table not in self._luts:
            from . import lut_from_table
            self._luts[table] = lut_from_table(self.N, SPACE, list(table), DELTA)
        return self._luts[table]

    # encodings
    def trivial(self, vals) -> np.ndarray:
        v = np.asarray(vals, dtype=np.uint64)
        out = np.zeros(v.shape + (self.dim,), dtype=np.uint64)
        with np.errstate(over="ignore"):
            out[..., -1] = (v % np.uint64(SPACE)) * np.uint64(DELTA)
        return out

    def bootstrap(self, reqs: Sequence[Tuple[np.ndarray, Tuple[int, ...]]]) -> List[np.ndarray]:
        shapes = [a.shape[:-1] for a, _ in reqs]
        if not reqs:
            return []
        tables = []
        index = {}
        idx_parts = []
        flat_parts = []
        for a, t in reqs:
            if t not in index:
                index[t] = len(tables)
                tables.append(t)
            cnt = int(np.prod(a.shape[:-1], dtype=np.int64))
            flat_parts.append(a.reshape(cnt, self.dim))
            idx_parts.append(np.full(cnt, index[t], dtype=np.uint32))
        flat = np.concatenate(flat_parts, axis=0)
        idx = np.concatenate(idx_parts)
        # one level = one launch; levels of wide operators (euint128 mul: ~10^5 PBS per operand pair) go in
        # chunks of MAX_LAUNCH ciphertexts so host and device staging stay bounded
        outs = [self._pbs(flat[o:o + MAX_LAUNCH], tables, idx[o:o + MAX_LAUNCH])
                for o in range(0, flat.shape[0], MAX_LAUNCH)]
        out = outs[0] if len(outs) == 1 else np.concatenate(outs, axis=0)
        self.pbs_count += flat.shape[0]
        self.launches += 1
        res, off = [], 0
        for s in shapes:
            cnt = int(np.prod(s, dtype=np.int64))
            res.append(out[off:off + cnt].reshape(s + (self.dim,)))
            off += cnt
        return res

    def _pbs(self, flat, tables, idx):
        luts = np.stack([self.lut(t) for t in tables])
        return self.engine.pbs(flat, luts, idx)

    def run(self, op):
        return self.run_many([op])[0]

    def run_many(self, ops) -> list:
        results = [None] * len(ops)
        pending = {}
        for i, g in enumerate(ops):
            try:
                pending[i] = (g, next(g))
            except StopIteration as e:
                results[i] = e.value
        while pending:
            order = list(pending)
            reqs, counts = [], []
            for i in order:
                reqs.extend(pending[i][1])
                counts.append(len(pending[i][1]))
            outs = self.bootstrap(reqs)
            off = 0
            for i, cnt in zip(order, counts):
                g = pending[i][0]
                try:
                    pending[i] = (g, g.send(outs[off:off + cnt]))
                except StopIteration as e:
                    results[i] = e.value
                    del pending[i]
                off += cnt
        return results


# --------------------------------------------------------------------------------------------
# linear operations on block arrays (mod 2^64, any leading shape)
# --------------------------------------------------------------------------------------------
def _add(*xs):
    with np.errstate(over="ignore"):
        out = xs[0].copy()
        for x in xs[1:]:
            out += x
    return out


def _scale(x, k: int):
    with np.errstate(over="ignore"):
        return (x * np.uint64(k % _M64)).astype(np.uint64)


def _const(c: "RadixCircuit", shape, v: int):
    return c.trivial(np.full(shape, v, dtype=np.uint64))


def _pack(x, y):
    """4x + y for clean blocks (the bivariate PBS input)."""
    return _add(_scale(x, MSG), y)


def _not(c, a):
    """3 - a for clean blocks (bitwise NOT of the 2-bit message), no PBS."""
    with np.errstate(over="ignore"):
        return (_const(c, a.shape[:-1], MSG - 1) - a).astype(np.uint64)


class RadixUint:
    """A batch of B encrypted w-bit integers: blocks (B, w/2, dim), LSB block first, all clean."""

    def __init__(self, c: RadixCircuit, blocks: np.ndarray):
        self.c, self.blocks = c, blocks

    @property
    def width(self) -> int:
        return 2 * self.blocks.shape[1]

    @property
    def batch(self) -> int:
        return self.blocks.shape[0]

    @staticmethod
    def _digits(values, w):
        """(B, w/2) base-4 digits, least significant first; values are ints of any size."""
        if w <= 64:
            v = np.atleast_1d(np.asarray(values, dtype=np.uint64))
            return (v[:, None] >> (2 * np.arange(w // 2, dtype=np.uint64))[None, :]) & np.uint64(3)
        vs = [int(x) for x in np.atleast_1d(np.asarray(values, dtype=object))]
        return np.array([[(x >> (2 * j)) & 3 for j in range(w // 2)] for x in vs], dtype=np.uint64).reshape(len(vs), w // 2)

    @classmethod
    def encrypt(cls, c: RadixCircuit, ck, values, w: int, seed: Optional[int] = None, stream0: int = 0) -> "RadixUint":
        d = cls._digits(values, w)
        ct = ck.encrypt(d.reshape(-1), SPACE, seed, stream0).reshape(d.shape + (-1,))
        return cls(c, ct)

    @classmethod
    def trivial(cls, c: RadixCircuit, values, w: int) -> "RadixUint":
        return cls(c, c.trivial(cls._digits(values, w)))

    def decrypt(self, ck) -> np.ndarray:
        B, nb = self.blocks.shape[:2]
        d = ck.decrypt(self.blocks.reshape(B * nb, -1), SPACE).reshape(B, nb).astype(object)
        w = self.width
        vals = [sum(int(d[i, j]) << (2 * j) for j in range(nb)) % (1 << w) for i in range(B)]
        return np.array(vals, dtype=np.uint64 if w <= 64 else object)

    def cast(self, w: int) -> "RadixUint":
        nb = w // 2
        if nb == self.blocks.shape[1]:
            return self
        if nb < self.blocks.shape[1]:
            return RadixUint(self.c, self.blocks[:, :nb])
        pad = _const(self.c, (self.batch, nb - self.blocks.shape[1]), 0)
        return RadixUint(self.c, np.concatenate([self.blocks, pad], axis=1))


# --------------------------------------------------------------------------------------------
# circuits (coroutines yielding levels of (lin, table))
# --------------------------------------------------------------------------------------------
T_MSG = _table(lambda v: v % MSG)
T_STATE = _table(lambda v: 2 if v >= MSG else (1 if v == MSG - 1 else 0))   # of a block sum <= 7
T_MERGE = _biv(lambda hi, lo: lo if hi == 1 else hi)                       # prefix op on states
T_APPLY = _biv(lambda st, m: (m + (1 if st == 2 else 0)) % MSG)            # carry-in from the prefix


def g_propagate(c: RadixCircuit, s: np.ndarray, carry_in: bool):
    """Carry propagation of block sums s (B, nb, dim) with values <= 7: clean result blocks."""
    B, nb = s.shape[:2]
    if carry_in:
        s = s.copy()
        s[:, 0] = _add(s[:, 0], _const(c, (B,), 1))
    msg, st = yield [(s, T_MSG), (s, T_STATE)]
    # Kogge-Stone over block states: prefix[j] = state of blocks 0..j
    d = 1
    while d < nb:
        (merged,) = yield [(_pack(st[:, d:], st[:, :-d]), T_MERGE)]
        st = np.concatenate([st[:, :d], merged], axis=1)
        d *= 2
    if nb == 1:
        return msg
    (hi,) = yield [(_pack(st[:, :-1], msg[:, 1:]), T_APPLY)]
    return np.concatenate([msg[:, :1], hi], axis=1)


def g_add(c, a, b, carry_in=False):
    return (yield from g_propagate(c, _add(a, b), carry_in))


def g_sub(c, a, b):
    return (yield from g_propagate(c, _add(a, _not(c, b)), True))


T_AND = _biv(lambda x, y: x & y)
T_OR = _biv(lambda x, y: x | y)
T_XOR = _biv(lambda x, y: x ^ y)
T_EQ = _biv(lambda x, y: int(x == y))
T_AND1 = _biv(lambda x, y: x & y & 1)
T_CMP = _biv(lambda x, y: 0 if x < y else (1 if x == y else 2))           # {<, =, >}
T_SEL_T = _biv(lambda cond, x: x if cond == 1 else 0)
T_SEL_F = _biv(lambda cond, x: 0 if cond == 1 else x)


def g_bitwise(c, kind, a, b):
    t = {"and": T_AND, "or": T_OR, "xor": T_XOR}[kind]
    (r,) = yield [(_pack(a, b), t)]
    return r


def g_eq(c, a, b):
    """encrypted bool block (B, dim), value 0/1."""
    (e,) = yield [(_pack(a, b), T_EQ)]
    while e.shape[1] > 1:
        if e.shape[1] % 2:
            e = np.concatenate([e, _const(c, (e.shape[0], 1), 1)], axis=1)
        (e,) = yield [(_pack(e[:, 0::2], e[:, 1::2]), T_AND1)]
    return e[:, 0]


def g_cmp(c, a, b):
    """comparison state of a vs b per value: block (B, dim) with 0 (<), 1 (=), 2 (>)."""
    (st,) = yield [(_pack(a, b), T_CMP)]
    # merge MSB-first: result = hi if hi != '=' else lo  (blocks are LSB first: hi = odd index)
    while st.shape[1] > 1:
        if st.shape[1] % 2:
            st = np.concatenate([st, _const(c, (st.shape[0], 1), 1)], axis=1)
        (st,) = yield [(_pack(st[:, 1::2], st[:, 0::2]), T_MERGE_CMP)]
    return st[:, 0]


T_MERGE_CMP = _biv(lambda hi, lo: lo if hi == 1 else hi)
T_IS = {"lt": _table(lambda v: int(v == 0)), "le": _table(lambda v: int(v <= 1)),
        "gt": _table(lambda v: int(v == 2)), "ge": _table(lambda v: int(v >= 1))}


def g_compare(c, kind, a, b):
    st = yield from g_cmp(c, a, b)
    (r,) = yield [(st, T_IS[kind])]
    return r


def g_select(c, cond, x, y):
    """cond (B, dim) in {0,1} ? x : y, blockwise: two bivariate PBS per block, then one message
    PBS of their sum, so the result is a fresh block again (noise level 1; a bivariate input 4x + y
    has level 5 = max_noise_level of the parameter set, so levels never stack)."""
    cw = np.broadcast_to(cond[:, None, :], x.shape)
    t, f = yield [(_pack(cw, x), T_SEL_T), (_pack(cw, y), T_SEL_F)]
    (r,) = yield [(_add(t, f), T_MSG)]
    return r


def g_minmax(c, kind, a, b):
    st = yield from g_cmp(c, a, b)
    (take_a,) = yield [(st, T_IS["lt"] if kind == "min" else T_IS["gt"])]
    return (yield from g_select(c, take_a, a, b))


T_SHL_LO = _biv(lambda cur, prev: ((cur << 1) | (prev >> 1)) & 3)   # one-bit left shift across blocks
T_SHR_LO = _biv(lambda nxt, cur: ((cur >> 1) | (nxt << 1)) & 3)     # one-bit right shift


def g_shift(c, a, k: int, kind: str):
    B, nb = a.shape[:2]
    w = 2 * nb
    k %= w
    q, r = divmod(k, 2)
    zero = _const(c, (B, q), 0)
    rot = kind in ("rotl", "rotr")
    if kind in ("shl", "rotl"):
        moved = np.roll(a, q, axis=1) if rot else np.concatenate([zero, a[:, :nb - q]], axis=1)
        if not r:
            return moved
        prev = np.roll(moved, 1, axis=1) if rot else np.concatenate([_const(c, (B, 1), 0), moved[:, :-1]], axis=1)
        (out,) = yield [(_pack(moved, prev), T_SHL_LO)]
        return out
    moved = np.roll(a, -q, axis=1) if rot else np.concatenate([a[:, q:], zero], axis=1)
    if not r:
        return moved
    nxt = np.roll(moved, -1, axis=1) if rot else np.concatenate([moved[:, 1:], _const(c, (B, 1), 0)], axis=1)
    (out,) = yield [(_pack(nxt, moved), T_SHR_LO)]
    return out


T_MUL_LO = _biv(lambda x, y: (x * y) % MSG)
T_MUL_HI = _biv(lambda x, y: (x * y) // MSG)
T_CARRY = _table(lambda v: v // MSG)


def g_sum_columns(c, cols: List[List[np.ndarray]], B: int):
    """Sum per-position lists of clean blocks (position k has weight 4^k, positions >= nb dropped)
    into one clean radix value: carry-save rounds add up to 5 blocks (<= 15, the block capacity) and
    split each sum into message (stays) and carry (moves up) in one PBS level, until every position
    holds at most two blocks; then one carry-propagating add."""
    nb = len(cols)
    while max(len(col) for col in cols) > 2:
        reqs, plan = [], []
        new_cols: List[List[np.ndarray]] = [[] for _ in range(nb)]
        for k, col in enumerate(cols):
            if len(col) <= 2:
                new_cols[k].extend(col)
                continue
            for g in range(0, len(col), 5):
                grp = col[g:g + 5]
                if len(grp) == 1:
                    new_cols[k].append(grp[0])
                    continue
                ssum = _add(*grp)
                reqs += [(ssum, T_MSG), (ssum, T_CARRY)]
                plan.append(k)
        outs = yield reqs
        for t, k in enumerate(plan):
            new_cols[k].append(outs[2 * t])
            if k + 1 < nb:
                new_cols[k + 1].append(outs[2 * t + 1])
        cols = new_cols
    zero = _const(c, (B,), 0)
    a = np.stack([col[0] if len(col) > 0 else zero for col in cols], axis=1)
    b = np.stack([col[1] if len(col) > 1 else zero for col in cols], axis=1)
    return (yield from g_add(c, a, b))


def g_mul(c, a, b):
    """a * b mod 2^w.  b: blocks (B, nb, dim) or a plaintext int.  Block products: two bivariate
    PBS (low / high digit of x*y) per pair i + j < nb (plaintext: univariate per a-block and digit)."""
    B, nb = a.shape[:2]
    reqs, pos = [], []
    if isinstance(b, (int, np.integer)):
        digs = [(int(b) >> (2 * j)) & 3 for j in range(nb)]
        for i in range(nb):
            for j in range(nb - i):
                d = digs[j]
                if d == 0:
                    continue
                reqs.append((a[:, i], _table(lambda v, d=d: (v * d) % MSG)))
                pos.append(i + j)
                if i + j + 1 < nb:
                    reqs.append((a[:, i], _table(lambda v, d=d: (v * d) // MSG)))
                    pos.append(i + j + 1)
    else:
        for i in range(nb):
            for j in range(nb - i):
                packed = _pack(a[:, i], b[:, j])
                reqs.append((packed, T_MUL_LO))
                pos.append(i + j)
                if i + j + 1 < nb:
                    reqs.append((packed, T_MUL_HI))
                    pos.append(i + j + 1)
    cols: List[List[np.ndarray]] = [[] for _ in range(nb)]
    if reqs:
        outs = yield reqs
        for o, k in zip(outs, pos):
            cols[k].append(o)
    return (yield from g_sum_columns(c, cols, B))


T_BIT = {k: _table(lambda v, k=k: (v >> k) & 1) for k in (0, 1)}


def g_shift_enc(c, a, amount, kind: str):
    """Shift / rotate by an encrypted amount (mod w): barrel shifter, one select per amount bit."""
    B, nb = a.shape[:2]
    w = 2 * nb
    nbits = max(1, (w - 1).bit_length())
    reqs = [(amount[:, k // 2], T_BIT[k % 2]) for k in range(nbits)]
    bits = yield reqs
    cur = a
    for k in range(nbits):
        moved = yield from g_shift(c, cur, 1 << k, kind)
        cur = yield from g_select(c, bits[k], moved, cur)
    return cur


T_LOW_BIT = _table(lambda v: v & 1)


def g_div_rem_scalar(c, a, d: int):
    """(a // d, a % d) for a plaintext divisor by multiply-high: with l = ceil(log2 d) and
    m = ceil(2^(w+l) / d) (w + 1 bits), floor(a * m / 2^(w+l)) = floor(a / d) for every a < 2^w
    (m*d - 2^(w+l) < d, so the error term a*(m*d - 2^(w+l)) / d < 2^(w+l) never crosses an integer).
    One constant multiply at width 2w + 2, a block shift, one constant multiply and one subtract.
    d = 0 follows tfhe-rs / fhEVM: quotient all ones, remainder = numerator.  Powers of two are a
    block shift and a mask."""
    B, nb = a.shape[:2]
    w = 2 * nb
    d = int(d) % (1 << w)
    if d == 0:
        return _const(c, (B, nb), MSG - 1), a
    if d & (d - 1) == 0:
        s = d.bit_length() - 1
        q = (yield from g_shift(c, a, s, "shr")) if s else a
        keep = s // 2
        parts = [a[:, :keep]]
        if s % 2:
            (lowbit,) = yield [(a[:, keep], T_LOW_BIT)]
            parts.append(lowbit[:, None])
        done = keep + s % 2
        parts.append(_const(c, (B, nb - done), 0))
        return q, np.concatenate(parts, axis=1)
    l = (d - 1).bit_length()
    m = -(-(1 << (w + l)) // d)
    nbw = w + 1                                             # width 2w + 2 holds a * m < 2^(2w+1)
    a_ext = np.concatenate([a, _const(c, (B, nbw - nb), 0)], axis=1)
    prod = yield from g_mul(c, a_ext, m)
    k = w + l
    sub = prod[:, k // 2:k // 2 + nb + 1]
    if sub.shape[1] < nb + 1:
        sub = np.concatenate([sub, _const(c, (B, nb + 1 - sub.shape[1]), 0)], axis=1)
    q = (yield from g_shift(c, sub, k % 2, "shr"))[:, :nb] if k % 2 else sub[:, :nb]
    qd = yield from g_mul(c, q, d)
    r = yield from g_sub(c, a, qd)
    return q, r


RADIX_OPS = ("add", "sub", "mul", "div", "rem", "and", "or", "xor", "eq", "ne", "lt", "le", "gt", "ge", "min", "max",
             "neg", "not", "shl", "shr", "rotl", "rotr")


def fhevm_op(c: RadixCircuit, op: str, lhs, rhs=None):
    """One fhEVM operator on radix integers (coroutine).  Comparisons return an encrypted bool block
    (B, dim) holding 0/1; other operators a RadixUint."""
    if op not in RADIX_OPS:
        raise ValueError(f"radix operator {op!r} not supported")
    if op == "not":
        return RadixUint(c, _not(c, lhs.blocks))
    if op == "neg":
        z = _const(c, lhs.blocks.shape[:-1], 0)
        return RadixUint(c, (yield from g_sub(c, z, lhs.blocks)))
    lenc, renc = isinstance(lhs, RadixUint), isinstance(rhs, RadixUint)
    if not (lenc or renc):
        raise ValueError("at least one operand must be encrypted")
    if op in ("shl", "shr", "rotl", "rotr"):
        if not lenc:
            raise ValueError("shift of a plaintext by an encrypted amount is not an fhEVM overload")
        if renc:
            return RadixUint(c, (yield from g_shift_enc(c, lhs.blocks, rhs.blocks, op)))
        return RadixUint(c, (yield from g_shift(c, lhs.blocks, int(rhs), op)))
    w = max(x.width for x in (lhs, rhs) if isinstance(x, RadixUint))
    B = (lhs if lenc else rhs).batch

    def blocks(x):
        if isinstance(x, RadixUint):
            return x.cast(w).blocks
        return c.trivial(np.broadcast_to(RadixUint._digits([int(x) % (1 << w)], w), (B, w // 2)))

    if op in ("div", "rem"):
        if not lenc or renc:
            raise ValueError("fhEVM div / rem take an encrypted numerator and a plaintext divisor")
        q, r = yield from g_div_rem_scalar(c, lhs.blocks, int(rhs))
        return RadixUint(c, q if op == "div" else r)
    if op == "mul":
        if not lenc:
            return RadixUint(c, (yield from g_mul(c, rhs.cast(w).blocks, int(lhs) % (1 << w))))
        if not renc:
            return RadixUint(c, (yield from g_mul(c, lhs.cast(w).blocks, int(rhs) % (1 << w))))
        return RadixUint(c, (yield from g_mul(c, blocks(lhs), blocks(rhs))))
    a, b = blocks(lhs), blocks(rhs)
    if op == "add":
        return RadixUint(c, (yield from g_add(c, a, b)))
    if op == "sub":
        return RadixUint(c, (yield from g_sub(c, a, b)))
    if op in ("and", "or", "xor"):
        return RadixUint(c, (yield from g_bitwise(c, op, a, b)))
    if op in ("eq", "ne"):
        e = yield from g_eq(c, a, b)
        if op == "eq":
            return e
        with np.errstate(over="ignore"):
            return (_const(c, e.shape[:-1], 1) - e).astype(np.uint64)
    if op in ("lt", "le", "gt", "ge"):
        return (yield from g_compare(c, op, a, b))
    return RadixUint(c, (yield from g_minmax(c, op, a, b)))
