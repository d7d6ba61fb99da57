"""Encrypted unsigned integers on the GPU gate bootstrap (the operator layer).

An encrypted w-bit integer is w gate-encoded bits (true = +1/8, false = -1/8 of the 2^64 torus,
LSB first) under the small LWE key.  Every gate is ONE keyswitch-PBS of a linear combination of
ciphertexts with the constant LUT 1/8 (TFHE gate bootstrapping); negation is free.

Operators are written as coroutines that ``yield`` one circuit LEVEL at a time (a list of arrays of
linear combinations) and receive the bootstrapped arrays back.  ``Circuit.run_many`` steps any
number of independent operator coroutines in lockstep and bootstraps the union of their levels in
one ``Engine.pbs`` launch, so a set of requests costs max(depth) launches, not sum(depth) — the
shape the GPU wants (a launch runs ~2k PBS in the time of one: SURVEY §8d).

Semantics follow the fhEVM Solidity operators whose KATs the reference replays
(tests/fhevm-suite/e2e/test/fhevmOperations*.ts, fixture tests/golden/fhevm_kats.json): wrapping
add/sub/mul mod 2^w, two's-complement neg, bitwise and/or/xor/not, comparisons to an encrypted
bool, unsigned min/max, shl/shr/rotl/rotr by (amount mod w), div/rem by a plaintext divisor
(x/0 = all-ones, x%0 = x as tfhe-rs), plaintext operands on either side, and mixed widths
zero-extended to the wider type.

Gates (inputs ±1/8; every |phase| stays <= 3/8 so no combination wraps past 1/2):
  AND  = PBS(a + b - 1/8)        OR  = PBS(a + b + 1/8)        XOR = PBS(2(a + b) + 1/4)
  MAJ  = PBS(a + b + c)          XOR3 = PBS(-2(a + b + c))     NOT = -a,  XNOR = -XOR
MAJ is the full-adder carry and also the parallel-prefix carry operator: with OR-type propagate
(P = carry-out given carry-in 1, G = given carry-in 0, so G implies P)
  (G, P)_hi o (G, P)_lo = (MAJ(G_hi, P_hi, G_lo), MAJ(G_hi, P_hi, P_lo)),
so a Kogge-Stone adder is 1 + log2(w) + 1 levels.  Small batches (latency-bound) use it; batches
that fill the GPU use the ripple adder (XOR3 + MAJ per bit, fewest PBS).
"""
from __future__ import annotations

from typing import Generator, List, Optional, Sequence, Union

import numpy as np

from . import MU, ClientKey, Engine

_M64 = 1 << 64
MAX_LAUNCH = 1 << 19  # ciphertexts per engine call (P-GATE: 2 x 631 x 8 B x 512 Ki = 5.3 GB of I/O)
WIDTHS = (8, 16, 32, 64, 128, 160, 256)   # ebool / euint* / eaddress of fhEVM (any width works)


# --------------------------------------------------------------------------------------------
# arrays: host numpy uint64, or (a device-resident Circuit) torch int64 tensors holding the same bits
# --------------------------------------------------------------------------------------------
def _is_t(a) -> bool:
    return type(a).__module__.startswith("torch")


def _cat(seq, axis: int = 0):
    seq = list(seq)
    if seq and _is_t(seq[0]):
        import torch
        return torch.cat(seq, dim=axis)
    return np.concatenate(seq, axis=axis)


def _stack(seq, axis: int = 0):
    seq = list(seq)
    if seq and _is_t(seq[0]):
        import torch
        return torch.stack(seq, dim=axis)
    return np.stack(seq, axis=axis)


def _bcast(a, shape):
    return a.expand(*shape) if _is_t(a) else np.broadcast_to(a, shape)


def _roll(a, k: int, axis: int):
    if _is_t(a):
        import torch
        return torch.roll(a, k, dims=axis)
    return np.roll(a, k, axis=axis)


def _where(mask: np.ndarray, x, y):
    """mask: host bools broadcasting against x / y."""
    if _is_t(x):
        import torch
        return torch.where(torch.as_tensor(np.ascontiguousarray(mask), device=x.device), x, y)
    return np.where(mask, x, y)


def _contig(a):
    return a.contiguous() if _is_t(a) else np.ascontiguousarray(a)


def _i64(v: int) -> int:
    v %= _M64
    return v - _M64 if v >= 1 << 63 else v


# --------------------------------------------------------------------------------------------
# linear combinations (all arithmetic mod 2^64, vectorised over any leading shape)
# --------------------------------------------------------------------------------------------
def _lin(terms, const: int = 0):
    """sum w * c + const on the body, mod 2^64, in one fresh array (weights +-1 as in-place adds / subtracts: the
    circuits' levels are tens of MB, so the host time between launches is these passes).  Device tensors: the
    same on int64 (two's-complement wrap-around = arithmetic mod 2^64)."""
    if _is_t(terms[0][1]):
        out = None
        for w, c in terms:
            w = _i64(w)
            t = c if w == 1 else -c if w == -1 else c * w
            out = (t.clone() if w == 1 else t) if out is None else out.add_(t)
        out[..., -1] += _i64(const)
        return out
    with np.errstate(over="ignore"):
        out = None
        for w, c in terms:
            w %= _M64
            if out is None:
                out = (np.array(c, dtype=np.uint64, copy=True) if w == 1 else
                       np.subtract(np.uint64(0), c, dtype=np.uint64) if w == _M64 - 1 else c * np.uint64(w))
            elif w == 1:
                np.add(out, c, out=out)
            elif w == _M64 - 1:
                np.subtract(out, c, out=out)
            else:
                np.add(out, c * np.uint64(w), out=out)
        out[..., -1] += np.uint64(const % _M64)
    return out


def AND(a, b):
    return _lin([(1, a), (1, b)], -MU)


def OR(a, b):
    return _lin([(1, a), (1, b)], MU)


def XOR(a, b):
    return _lin([(2, a), (2, b)], 2 * MU)


def MAJ(a, b, c):
    return _lin([(1, a), (1, b), (1, c)])


def XOR3(a, b, c):
    return _lin([(-2, a), (-2, b), (-2, c)])


def NOT(a):
    if _is_t(a):
        return -a
    with np.errstate(over="ignore"):
        return np.subtract(np.uint64(0), a, dtype=np.uint64)


# --------------------------------------------------------------------------------------------
# lockstep scheduler
# --------------------------------------------------------------------------------------------
Level = List[np.ndarray]
Op = Generator[Level, List[np.ndarray], object]


class Circuit:
    """Runs operator coroutines on an Engine: every yielded level is one batched PBS launch."""

    def __init__(self, engine: Engine, capacity: int = 2048, round_size: Optional[int] = None, device=None):
        self.engine = engine
        self.dim = engine.params.n + 1
        self.lut = engine.gate_lut()
        # device-resident circuit (a torch device, e.g. "cuda:0"): ciphertexts are int64 tensors on it, every
        # level is one Engine.pbs_device launch on torch's current stream and the linear combinations are torch
        # ops queued behind it -- no host round trip per level (the host only walks the circuit's structure)
        self.device = device
        if device is not None:
            import torch
            self._lut_d = None if self.lut is None else torch.from_numpy(self.lut.view(np.int64).copy()).to(device)
        self.capacity = capacity      # PBS one launch completes in ~one PBS latency (8 x 256 CUs)
        # PBS per round of the engine's batch kernel (Engine.round_size: the FFT64 pair kernel holds 4
        # ciphertexts x 256 CUs per GPU); a launch of n PBS costs ~max(1, ceil(n / round_size)) rounds -- the
        # carry-out circuit's cost model.  Engines without the property (test doubles) model one P-GATE GPU.
        self.round_size = round_size or getattr(engine, "round_size", 1024)
        self.pbs_count = 0
        self.launches = 0

    def trivial(self, bits) -> np.ndarray:
        """Noise-free encryptions (0, ..., 0, ±1/8) of clear bits (plaintext operands)."""
        bits = np.asarray(bits, dtype=bool)
        out = np.zeros(bits.shape + (self.dim,), dtype=np.uint64)
        out[..., -1] = np.where(bits, np.uint64(MU), np.uint64(_M64 - MU))
        return out if self.device is None else self.to_device(out)

    def to_device(self, a):
        """Host uint64 array -> this circuit's arrays (a device tensor in device mode)."""
        if self.device is None or _is_t(a):
            return a
        import torch
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(self.device)

    def bootstrap(self, lins: Sequence[np.ndarray]) -> List[np.ndarray]:
        shapes = [tuple(l.shape[:-1]) for l in lins]
        if self.device is not None:
            return self._bootstrap_device(lins, shapes)
        flat = np.concatenate([l.reshape(-1, self.dim) for l in lins], axis=0) if lins else \
            np.zeros((0, self.dim), np.uint64)
        if flat.shape[0]:
            # one level = one launch, in chunks of MAX_LAUNCH ciphertexts (euint128 mul levels reach ~10^6)
            outs = [self.engine.pbs(flat[o:o + MAX_LAUNCH], self.lut) for o in range(0, flat.shape[0], MAX_LAUNCH)]
            out = outs[0] if len(outs) == 1 else np.concatenate(outs, axis=0)
            self.pbs_count += flat.shape[0]
            self.launches += 1
        else:
            out = flat
        res, off = [], 0
        for s in shapes:
            cnt = int(np.prod(s, dtype=np.int64))
            res.append(out[off:off + cnt].reshape(s + (self.dim,)))
            off += cnt
        return res

    def _bootstrap_device(self, lins, shapes):
        import torch
        flat = torch.cat([l.reshape(-1, self.dim) for l in lins], dim=0) if lins else \
            torch.zeros((0, self.dim), dtype=torch.int64, device=self.device)
        if flat.shape[0]:
            outs = [self.engine.pbs_device(flat[o:o + MAX_LAUNCH], self._lut_d)
                    for o in range(0, flat.shape[0], MAX_LAUNCH)]
            out = outs[0] if len(outs) == 1 else torch.cat(outs, dim=0)
            self.pbs_count += flat.shape[0]
            self.launches += 1
        else:
            out = flat
        res, off = [], 0
        for sh in shapes:
            cnt = int(np.prod(sh, dtype=np.int64))
            res.append(out[off:off + cnt].reshape(sh + (self.dim,)))
            off += cnt
        return res

    def run(self, op: Op):
        return self.run_many([op])[0]

    def run_many(self, ops: Sequence[Op]) -> list:
        results = [None] * len(ops)
        pending = {}
        for i, g in enumerate(ops):
            try:
                pending[i] = (g, next(g))
            except StopIteration as e:
                results[i] = e.value
        while pending:
            order = list(pending)
            lins, counts = [], []
            for i in order:
                lvl = pending[i][1]
                lins.extend(lvl)
                counts.append(len(lvl))
            outs = self.bootstrap(lins)
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

    def prefer_prefix(self, batch: int, width: int) -> bool:
        """Latency-bound (the level's PBS fit in one launch wave) -> log-depth prefix adder."""
        return batch * width * 2 <= self.capacity

    def carry_block(self, batch: int, width: int) -> int:
        """Block size of the carry-out circuit (_carry_out) with the fewest launch rounds (then the
        fewest PBS): s = width is the ripple chain, s = 1 the bit-level reduction tree."""
        best = None
        for s in sorted({1 << k for k in range(width.bit_length())} | {width}):
            if s > width:
                continue
            lv = _carry_levels(batch, width, s)
            key = (sum(max(1, -(-n // self.round_size)) for n in lv), sum(lv), -s)
            if best is None or key < best[0]:
                best = (key, s)
        return best[1]


# --------------------------------------------------------------------------------------------
# bit-vector circuits: arrays of shape (B, w, dim), LSB first
# --------------------------------------------------------------------------------------------
def _zeros(c: Circuit, B: int, w: int) -> np.ndarray:
    return c.trivial(np.zeros((B, w), dtype=bool))


def g_bitwise(kind: str, a: np.ndarray, b: np.ndarray) -> Op:
    gate = {"and": AND, "or": OR, "xor": XOR}[kind]
    (r,) = yield [gate(a, b)]
    return r


def g_add(c: Circuit, a: np.ndarray, b: np.ndarray, cin: bool = False, want_sum: bool = True,
          want_carry: bool = False, prefix: bool = None) -> Op:
    """a + b + cin over w bits.  Returns (sum bits or None, carry-out or None)."""
    B, w = a.shape[0], a.shape[1]
    if not want_sum:
        # only the carry-out (comparisons): block ripple + reduction tree, block size by the cost model
        s = c.carry_block(B, w) if prefix is None else (1 if prefix else w)
        return None, (yield from _carry_out(c, a, b, cin, s))
    if prefix is None:
        prefix = c.prefer_prefix(B, w)
    if not prefix:
        carry = c.trivial(np.full((B,), cin, dtype=bool))
        sums = []
        for i in range(w):
            lvl = []
            need_carry = i < w - 1 or want_carry
            if need_carry:
                lvl.append(MAJ(a[:, i], b[:, i], carry))
            if want_sum:
                lvl.append(XOR3(a[:, i], b[:, i], carry))
            out = yield lvl
            if want_sum:
                sums.append(out[-1])
            if need_carry:
                carry = out[0]
        return (_stack(sums, axis=1) if want_sum else None), (carry if want_carry else None)
    # Kogge-Stone: inclusive prefixes (G, P)[0..i]
    G, P = yield [AND(a, b), OR(a, b)]
    d = 1
    while d < w:
        hi_G, hi_P = G[:, d:], P[:, d:]
        nG, nP = yield [MAJ(hi_G, hi_P, G[:, :-d]), MAJ(hi_G, hi_P, P[:, :-d])]
        G = _cat([G[:, :d], nG], axis=1)
        P = _cat([P[:, :d], nP], axis=1)
        d *= 2
    pref = P if cin else G
    carries = _cat([c.trivial(np.full((B, 1), cin, dtype=bool)), pref[:, :w - 1]], axis=1)
    (s,) = yield [XOR3(a, b, carries)]
    return s, (pref[:, w - 1] if want_carry else None)


def _carry_levels(B: int, w: int, s: int) -> List[int]:
    """PBS per launch of _carry_out(width w, block size s) over a batch of B."""
    nb = -(-w // s)
    lv = [B * (1 + 2 * sum(1 for k in range(1, nb) if k * s + j < w)) for j in range(s)]
    n = nb
    while n > 1:
        lv.append(B * (1 + 2 * (n // 2 - 1)))
        n = n - n // 2
    return lv


def _carry_out(c: Circuit, a: np.ndarray, b: np.ndarray, cin: bool, s: int) -> Op:
    """Carry-out of a + b + cin over w bits (B, w, dim) in blocks of s bits: every block ripples its
    carries in lockstep with the others (block 0 from the known carry-in: one MAJ per bit; blocks k >= 1
    for both carry-ins, G = given 0 and P = given 1: AND / OR at their first bit, then two MAJ per bit),
    then a reduction tree merges neighbours, (G, P)_hi o (G, P)_lo = (MAJ(G_hi, P_hi, G_lo),
    MAJ(G_hi, P_hi, P_lo)) and C = MAJ(G_hi, P_hi, C_lo) onto block 0 (G implies P, so MAJ selects).
    s + ceil(log2(w / s)) levels: s = w is the ripple chain, s = 1 the bit-level tree."""
    B, w = a.shape[0], a.shape[1]
    nb = -(-w // s)
    C = c.trivial(np.full((B,), cin, dtype=bool))
    G = P = None                                   # (B, nb - 1, dim): blocks 1 .. nb - 1
    for j in range(s):
        ks = [k for k in range(1, nb) if k * s + j < w]
        lvl = [MAJ(a[:, j], b[:, j], C)]
        if ks:
            bits = [k * s + j for k in ks]
            ab, bb = a[:, bits], b[:, bits]
            if j == 0:
                lvl += [AND(ab, bb), OR(ab, bb)]
            else:
                m = len(ks)                        # the active blocks are 1 .. m (only the last can end early)
                lvl += [MAJ(ab, bb, G[:, :m]), MAJ(ab, bb, P[:, :m])]
        out = yield lvl
        C = out[0]
        if ks:
            if j == 0:
                G, P = out[1], out[2]
            else:
                G = _cat([out[1], G[:, len(ks):]], axis=1)
                P = _cat([out[2], P[:, len(ks):]], axis=1)
    while G is not None and G.shape[1] > 0:
        # states: C (block 0), then (G, P) of blocks 1 .. n-1; merge (0, 1) and (2i, 2i+1)
        n = G.shape[1] + 1
        npairs = n // 2 - 1                        # merges among blocks >= 2: (2, 3), (4, 5), ...
        lvl = [MAJ(G[:, 0], P[:, 0], C)]
        if npairs:
            hiG, hiP = G[:, 2:2 * npairs + 1:2], P[:, 2:2 * npairs + 1:2]
            loG, loP = G[:, 1:2 * npairs:2], P[:, 1:2 * npairs:2]
            lvl += [MAJ(hiG, hiP, loG), MAJ(hiG, hiP, loP)]
        out = yield lvl
        C = out[0]
        nG = [out[1]] if npairs else []
        nP = [out[2]] if npairs else []
        if n % 2:                                  # an odd block at the top passes through
            nG.append(G[:, n - 2:n - 1])
            nP.append(P[:, n - 2:n - 1])
        G = _cat(nG, axis=1) if nG else None
        P = _cat(nP, axis=1) if nP else None
    return C


def g_sub(c: Circuit, a, b, want_sum=True, want_carry=False) -> Op:
    """a - b = a + ~b + 1; carry-out = (a >= b)."""
    return (yield from g_add(c, a, NOT(b), True, want_sum, want_carry))


def g_ge(c: Circuit, a, b) -> Op:
    _, cout = yield from g_add(c, a, NOT(b), True, want_sum=False, want_carry=True)
    return cout


def g_eq(c: Circuit, a, b) -> Op:
    (x,) = yield [XOR(a, b)]
    cur = NOT(x)                                    # XNOR per bit
    B = a.shape[0]
    while cur.shape[1] > 1:
        if cur.shape[1] % 2:
            cur = _cat([cur, NOT(_zeros(c, B, 1))], axis=1)
        (cur,) = yield [AND(cur[:, 0::2], cur[:, 1::2])]
    return cur[:, 0]


def g_select(cond: np.ndarray, x: np.ndarray, y: np.ndarray) -> Op:
    """cond ? x : y bitwise in ONE level: t = AND(cond, x), f = AND(NOT cond, y), and since at most one of
    them is true, OR(t, f) = t + f + 1/8 holds exactly on the phases (-1/8 - 1/8 + 1/8 = -1/8, 1/8 - 1/8 + 1/8
    = 1/8): the OR needs no bootstrap.  The result carries the noise of two PBS outputs, still far inside
    the 1/8 decision margin of any gate it feeds.  Invariant: every consumer bootstraps it -- a select output
    never enters another non-bootstrapped linear combination (tests/test_gpu_select_noise.py measures the
    worst consumers, MAJ and XOR / XOR3 of select outputs, against their margins)."""
    cw = _bcast(cond[:, None, :], x.shape)
    t, f = yield [AND(cw, x), _lin([(-1, cw), (1, y)], -MU)]      # AND(cw, x), AND(NOT cw, y)
    return OR(t, f)


def g_mul(c: Circuit, a: np.ndarray, b: Union[np.ndarray, int], prefix=None) -> Op:
    """a * b mod 2^w: partial products (one level; none when b is plaintext), carry-save 3:2
    compression (XOR3 + MAJ: one level per layer), final adder."""
    B, w = a.shape[0], a.shape[1]
    rows = []
    if isinstance(b, (int, np.integer)):
        k = int(b) % (1 << w)
        for j in range(w):
            if (k >> j) & 1:
                rows.append(_cat([_zeros(c, B, j), a[:, :w - j]], axis=1))
    else:
        lvl = [AND(a[:, :w - j], _bcast(b[:, j:j + 1], (B, w - j, c.dim))) for j in range(w)]
        pp = yield lvl
        rows = [_cat([_zeros(c, B, j), pp[j]], axis=1) for j in range(w)]
    if not rows:
        return _zeros(c, B, w)
    while len(rows) > 2:
        ntrip = len(rows) // 3
        lvl = []
        for t in range(ntrip):
            x, y, z = rows[3 * t:3 * t + 3]
            lvl += [XOR3(x, y, z), MAJ(x[:, :w - 1], y[:, :w - 1], z[:, :w - 1])]
        out = yield lvl
        nrows = []
        for t in range(ntrip):
            nrows.append(out[2 * t])
            nrows.append(_cat([_zeros(c, B, 1), out[2 * t + 1]], axis=1))
        rows = nrows + rows[3 * ntrip:]
    if len(rows) == 1:
        return rows[0]
    s, _ = yield from g_add(c, rows[0], rows[1], prefix=prefix)
    return s


def g_div_rem_scalar(c: Circuit, a: np.ndarray, d: int) -> Op:
    """Restoring division by a plaintext divisor: returns (quotient, remainder)."""
    B, w = a.shape[0], a.shape[1]
    d = int(d) % (1 << w)
    if d == 0:  # tfhe-rs / fhEVM: quotient all ones, remainder = numerator
        return NOT(_zeros(c, B, w)), a
    L = d.bit_length()
    q = _zeros(c, B, w)
    # after shifting in the top k bits, R = a[w-k:] ; while k < L, R < d so q bits are 0
    k0 = L - 1
    R = a[:, w - k0:] if k0 > 0 else _zeros(c, B, 0)   # R has k0 bits
    for i in range(w - L, -1, -1):
        R = _cat([a[:, i:i + 1], R], axis=1)         # (R << 1) | a_i  : L..w bits
        r = R.shape[1]
        dbits = c.trivial(np.broadcast_to(np.array([(d >> j) & 1 for j in range(r)], dtype=bool), (B, r)))
        t, ge = yield from g_add(c, R, NOT(dbits), True, want_sum=True, want_carry=True)
        q[:, i] = ge
        R = yield from g_select(ge, t, R)
        R = R[:, :max(L, 1)] if r > L else R                   # R < d < 2^L after the step
    rem = _cat([R, _zeros(c, B, w - R.shape[1])], axis=1) if R.shape[1] < w else R[:, :w]
    return q, rem


def _shift_clear(c: Circuit, a: np.ndarray, k: int, kind: str) -> np.ndarray:
    B, w = a.shape[0], a.shape[1]
    k %= w
    if kind == "shl":
        return _cat([_zeros(c, B, k), a[:, :w - k]], axis=1)
    if kind == "shr":
        return _cat([a[:, k:], _zeros(c, B, k)], axis=1)
    if kind == "rotl":
        return _roll(a, k, 1)
    if kind == "rotr":
        return _roll(a, -k, 1)
    raise ValueError(kind)


def g_shift(c: Circuit, a: np.ndarray, amount: Union[np.ndarray, int], kind: str) -> Op:
    """Shift / rotate by (amount mod w): a plaintext amount is rewiring (free); an encrypted one
    is a barrel shifter, one select level per amount bit."""
    if isinstance(amount, (int, np.integer)):
        return _shift_clear(c, a, int(amount), kind)
    w = a.shape[1]
    cur = a
    for k in range((w - 1).bit_length()):
        cur = yield from g_select(amount[:, k], _shift_clear(c, cur, 1 << k, kind), cur)
    return cur


# --------------------------------------------------------------------------------------------
# typed values and the fhEVM operator dispatch
# --------------------------------------------------------------------------------------------
class FheUint:
    """A batch of B encrypted w-bit unsigned integers: ``bits`` is (B, w, n+1), LSB first."""

    def __init__(self, circuit: Circuit, bits: np.ndarray):
        self.c, self.bits = circuit, bits

    @property
    def width(self) -> int:
        return self.bits.shape[1]

    @property
    def batch(self) -> int:
        return self.bits.shape[0]

    @staticmethod
    def _bits_of(values, width: int) -> np.ndarray:
        """(B, width) bool, LSB first; values are ints of any size (euint64/128/256 and wider)."""
        if width <= 64:
            v = np.atleast_1d(np.asarray(values, dtype=np.uint64))
            return ((v[:, None] >> np.arange(width, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
        vs = [int(x) for x in np.atleast_1d(np.asarray(values, dtype=object))]
        return np.array([[(x >> j) & 1 for j in range(width)] for x in vs], dtype=bool).reshape(len(vs), width)

    @classmethod
    def encrypt(cls, circuit: Circuit, ck: ClientKey, values, width: int, seed: Optional[int] = None,
                stream0: int = 0) -> "FheUint":
        b = cls._bits_of(values, width)
        ct = ck.encrypt_bool(b.reshape(-1), seed, stream0).reshape(b.shape[0], width, -1)
        return cls(circuit, circuit.to_device(ct))

    @classmethod
    def trivial(cls, circuit: Circuit, values, width: int) -> "FheUint":
        return cls(circuit, circuit.trivial(cls._bits_of(values, width)))

    def decrypt(self, ck: ClientKey) -> np.ndarray:
        return decrypt_bits(ck, self.bits)

    def cast(self, width: int) -> "FheUint":
        """Zero-extend / truncate."""
        if width == self.width:
            return self
        if width < self.width:
            return FheUint(self.c, self.bits[:, :width])
        return FheUint(self.c, _cat([self.bits, _zeros(self.c, self.batch, width - self.width)], 1))

    # synchronous operator sugar (each call runs its own levels; use Circuit.run_many + fhevm_op
    # to batch independent operations)
    def _r(self, op):
        return self.c.run(op)

    def __add__(self, o):
        return FheUint(self.c, self._r(fhevm_op(self.c, "add", self, o)).bits)

    def __sub__(self, o):
        return FheUint(self.c, self._r(fhevm_op(self.c, "sub", self, o)).bits)

    def __mul__(self, o):
        return FheUint(self.c, self._r(fhevm_op(self.c, "mul", self, o)).bits)

    def __and__(self, o):
        return self._r(fhevm_op(self.c, "and", self, o))

    def __or__(self, o):
        return self._r(fhevm_op(self.c, "or", self, o))

    def __xor__(self, o):
        return self._r(fhevm_op(self.c, "xor", self, o))

    def __neg__(self):
        return self._r(fhevm_op(self.c, "neg", self))

    def __invert__(self):
        return FheUint(self.c, NOT(self.bits))

    def op(self, name: str, other=None):
        return self._r(fhevm_op(self.c, name, self, other))


def decrypt_bits(ck: ClientKey, bits: np.ndarray) -> np.ndarray:
    """(B,) uint64 for w <= 64; an object array of Python ints for wider values."""
    if _is_t(bits):
        bits = bits.cpu().numpy().view(np.uint64)
    B, w = bits.shape[0], bits.shape[1]
    b = ck.decrypt_bool(bits.reshape(-1, bits.shape[-1])).reshape(B, w)
    if w <= 64:
        b = b.astype(np.uint64)
        return (b << np.arange(w, dtype=np.uint64)[None, :]).sum(axis=1).astype(np.uint64)
    return np.array([sum(1 << j for j in range(w) if row[j]) for row in b], dtype=object)


BINARY_OPS = ("add", "sub", "mul", "div", "rem", "and", "or", "xor", "shl", "shr", "rotl", "rotr",
              "eq", "ne", "ge", "gt", "le", "lt", "min", "max")
UNARY_OPS = ("neg", "not")
BOOL_RESULT = ("eq", "ne", "ge", "gt", "le", "lt")


def fhevm_op(c: Circuit, op: str, lhs, rhs=None) -> Op:
    """One fhEVM operator as a coroutine.  ``lhs``/``rhs`` are FheUint or plaintext ints (at most
    one plaintext); mixed widths widen to the larger (fhevm TFHE.sol overloads).  Returns a
    FheUint, or for comparisons an encrypted bool array of shape (B, n+1)."""
    if op in UNARY_OPS:
        a = lhs.bits
        if op == "not":
            return FheUint(c, NOT(a))
        s, _ = yield from g_sub(c, _zeros(c, a.shape[0], a.shape[1]), a)
        return FheUint(c, s)
    if op not in BINARY_OPS:
        raise ValueError(f"unknown operator {op!r}")
    l_enc, r_enc = isinstance(lhs, FheUint), isinstance(rhs, FheUint)
    if not (l_enc or r_enc):
        raise ValueError("at least one operand must be encrypted")
    if op in ("shl", "shr", "rotl", "rotr"):
        if not l_enc:
            raise ValueError("shift of a plaintext by an encrypted amount is not an fhEVM overload")
        if r_enc:
            nb = max(1, (lhs.width - 1).bit_length())
            amt = rhs.bits if rhs.width >= nb else rhs.cast(nb).bits
        else:
            amt = int(rhs)
        return FheUint(c, (yield from g_shift(c, lhs.bits, amt, op)))
    if op in ("div", "rem"):
        if not l_enc or r_enc:
            raise ValueError("div/rem take an encrypted numerator and a plaintext divisor")
        q, r = yield from g_div_rem_scalar(c, lhs.bits, int(rhs))
        return FheUint(c, q if op == "div" else r)
    w = max(x.width for x in (lhs, rhs) if isinstance(x, FheUint))
    B = (lhs if l_enc else rhs).batch

    def bits(x):
        return x.cast(w).bits if isinstance(x, FheUint) else c.trivial(
            np.broadcast_to(FheUint._bits_of([int(x) % (1 << w)], w), (B, w)))

    if op == "mul":
        if not l_enc:
            return FheUint(c, (yield from g_mul(c, rhs.cast(w).bits, int(lhs))))
        if not r_enc:
            return FheUint(c, (yield from g_mul(c, lhs.cast(w).bits, int(rhs))))
        return FheUint(c, (yield from g_mul(c, bits(lhs), bits(rhs))))
    a, b = bits(lhs), bits(rhs)
    if op in ("and", "or", "xor"):
        return FheUint(c, (yield from g_bitwise(op, a, b)))
    if op == "add":
        s, _ = yield from g_add(c, a, b)
        return FheUint(c, s)
    if op == "sub":
        s, _ = yield from g_sub(c, a, b)
        return FheUint(c, s)
    if op in ("eq", "ne"):
        e = yield from g_eq(c, a, b)
        return e if op == "eq" else NOT(e)
    if op in ("ge", "lt"):
        g = yield from g_ge(c, a, b)
        return g if op == "ge" else NOT(g)
    if op in ("le", "gt"):
        g = yield from g_ge(c, b, a)
        return g if op == "le" else NOT(g)
    # min / max
    lt = NOT((yield from g_ge(c, a, b)))
    if op == "min":
        return FheUint(c, (yield from g_select(lt, a, b)))
    return FheUint(c, (yield from g_select(lt, b, a)))
