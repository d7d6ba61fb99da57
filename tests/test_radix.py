"""Radix integers on P-FHEVM (tfhe_amd/radix.py) on CPU: circuit logic with a cleartext double of the
programmable bootstrap that evaluates the 16-entry tables on trivial blocks (and asserts that no
block ever reaches the padding bit), replaying the reference's fhEVM operator KATs for every
operator the radix layer implements.  The MI355X run is tests/test_gpu_radix.py."""
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest

from tfhe_amd import radix as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "fhevm_kats.json")


class CleartextRadixCircuit(R.RadixCircuit):
    def __init__(self, N=2048):
        # trivial blocks: the mask width does not matter (N=2 keeps the euint128 levels in memory)
        eng = SimpleNamespace(params=SimpleNamespace(k=1, N=N, n=918, order=1))
        super().__init__(eng)
        self.max_seen = 0

    def _pbs(self, flat, tables, idx):
        assert not flat[:, :-1].any(), "trivial blocks only"
        v = (flat[:, -1] // np.uint64(R.DELTA)).astype(np.int64)
        assert np.all(flat[:, -1] % np.uint64(R.DELTA) == 0)
        assert v.max(initial=0) < R.SPACE, f"block value {v.max()} crossed the padding bit"
        self.max_seen = max(self.max_seen, int(v.max(initial=0)))
        out = np.array([tables[i][x] for i, x in zip(idx, v)], dtype=np.uint64)
        return self.trivial(out)


class ClearKey:
    def decrypt(self, cts, mm):
        return (np.asarray(cts)[..., -1] // np.uint64(R.DELTA)) % np.uint64(mm)


def _w(t):
    return 1 if t == "ebool" else int(t.lstrip("e").replace("uint", ""))


def kat_op(c, k):
    args = []
    for t, v in zip(k["types"], k["args"]):
        args.append(R.RadixUint.trivial(c, [v], _w(t)) if t.startswith("e") else int(v))
    return R.fhevm_op(c, k["op"], *args)


def check(ck, k, r):
    if k["result_type"] == "ebool":
        return int(ck.decrypt(r, R.SPACE)[0]) == int(bool(k["expect"]))
    return int(r.decrypt(ck)[0]) == k["expect"] and r.width == _w(k["result_type"])


def supported(k):
    return k["op"] in R.RADIX_OPS         # every fhEVM operator


@pytest.fixture(scope="module")
def kats():
    from conftest import load_kats
    return [k for k in load_kats() if supported(k)]


def test_radix_kats_cleartext(kats):
    assert len(kats) == 2394
    c = CleartextRadixCircuit(N=2)
    ck = ClearKey()
    res = c.run_many([kat_op(c, k) for k in kats])
    bad = [(k["source"], k["op"], k["args"], k["expect"]) for k, r in zip(kats, res) if not check(ck, k, r)]
    assert not bad, bad[:5]
    assert c.launches <= 40, c.launches
    assert c.max_seen <= 15


@pytest.mark.parametrize("w", [8, 32])
def test_radix_random_batch(w):
    rng = np.random.default_rng(w)
    B = 50
    a = rng.integers(0, 1 << w, B, dtype=np.uint64)
    b = rng.integers(0, 1 << w, B, dtype=np.uint64)
    b[:5] = a[:5]
    c = CleartextRadixCircuit()
    ck = ClearKey()
    A, Bv = R.RadixUint.trivial(c, a, w), R.RadixUint.trivial(c, b, w)
    ops = ["add", "sub", "xor", "lt", "ge", "eq", "min", "max", "neg", "mul"]
    res = c.run_many([R.fhevm_op(c, op, A, None if op == "neg" else Bv) for op in ops])
    m = (1 << w) - 1
    want = {"add": (a + b) & np.uint64(m), "sub": (a - b) & np.uint64(m), "xor": a ^ b, "lt": a < b, "ge": a >= b,
            "eq": a == b, "min": np.minimum(a, b), "max": np.maximum(a, b), "neg": (np.uint64(0) - a) & np.uint64(m),
            "mul": (a * b) & np.uint64(m)}
    for op, r in zip(ops, res):
        got = ck.decrypt(r, R.SPACE).astype(bool) if op in ("lt", "ge", "eq") else r.decrypt(ck)
        np.testing.assert_array_equal(got, want[op], err_msg=op)
    for k in (0, 1, 5, 13, 31):
        for kind in ("shl", "shr", "rotl", "rotr"):
            r = c.run(R.fhevm_op(c, kind, A, k))
            kk = k % w
            v = [int(x) for x in a]
            exp = {"shl": [(x << kk) & m for x in v], "shr": [x >> kk for x in v],
                   "rotl": [((x << kk) | (x >> (w - kk))) & m for x in v],
                   "rotr": [((x >> kk) | (x << (w - kk))) & m for x in v]}[kind]
            np.testing.assert_array_equal(r.decrypt(ck), np.array(exp, dtype=np.uint64), err_msg=f"{kind} {k}")


@pytest.mark.parametrize("w,divisors", [(8, [0, 1, 2, 3, 7, 8, 76, 128, 180, 255]),
                                         (32, [5, 550954323, 1 << 31, (1 << 32) - 1])])
def test_radix_div_rem_scalar(w, divisors):
    """multiply-high division against // and % (exhaustive numerators at w=8, edge values at w=32);
    d = 0 gives quotient all ones and remainder = numerator (tfhe-rs / fhEVM)."""
    rng = np.random.default_rng(w)
    m = (1 << w) - 1
    a = np.arange(256, dtype=np.uint64) if w == 8 else np.concatenate(
        [np.array([0, 1, m, m - 1, 550954323, 550954322], dtype=np.uint64), rng.integers(0, 1 << w, 40, dtype=np.uint64)])
    c = CleartextRadixCircuit()
    ck = ClearKey()
    A = R.RadixUint.trivial(c, a, w)
    res = c.run_many([R.fhevm_op(c, op, A, d) for d in divisors for op in ("div", "rem")])
    for t, d in enumerate(divisors):
        q, r = res[2 * t].decrypt(ck), res[2 * t + 1].decrypt(ck)
        wq = np.full_like(a, m) if d == 0 else a // np.uint64(d)
        wr = a if d == 0 else a % np.uint64(d)
        np.testing.assert_array_equal(q, wq, err_msg=f"div {d}")
        np.testing.assert_array_equal(r, wr, err_msg=f"rem {d}")
    assert c.max_seen <= 15
