"""Integer operator layer (tfhe_amd/integer.py) on CPU: circuit logic + phase margins.

The engine here is a test double that only accepts TRIVIAL ciphertexts (mask = 0), so a gate's
phase is its body: it checks every bootstrapped linear combination keeps >= 1/16 of the torus
away from the decision boundaries (0 and 1/2) and returns the trivial encryption of the gate
output.  The real GPU path replays the same KATs in tests/test_fhevm_kats.py (-m gpu).
KATs: tests/golden/fhevm_kats.json, extracted from the reference's
tests/fhevm-suite/e2e/test/fhevmOperations*.ts by tests/golden/extract_fhevm_kats.py.
"""
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest

from tfhe_amd import MU
from tfhe_amd import integer as I

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "fhevm_kats.json")
M64 = 1 << 64


class CleartextEngine:
    """Gate bootstrap on trivial ciphertexts: sign of the body (test double, CPU only)."""

    def __init__(self, n=630):
        self.params = SimpleNamespace(n=n, N=1024)
        self.min_margin = 1 << 62

    def gate_lut(self):
        return None

    def pbs(self, cts, lut):
        cts = np.asarray(cts, dtype=np.uint64)
        assert not cts[:, :-1].any(), "cleartext engine expects trivial ciphertexts"
        body = cts[:, -1]
        d0 = np.minimum(body, np.uint64(0) - body)                    # distance to 0
        half = np.uint64(1 << 63)
        d1 = np.minimum(body - half, half - body)                     # distance to 1/2
        margin = int(np.minimum(d0, d1).min()) if len(body) else 1 << 62
        self.min_margin = min(self.min_margin, margin)
        out = np.zeros_like(cts)
        pos = (body != 0) & (body < half)
        out[:, -1] = np.where(pos, np.uint64(MU), np.uint64(M64 - MU))
        return out


class ClearKey:
    def decrypt_bool(self, cts):
        b = np.asarray(cts, dtype=np.uint64)[..., -1]
        return (b != 0) & (b < np.uint64(1 << 63))


def _width(t):
    return 1 if t == "ebool" else int(t.lstrip("e").replace("uint", ""))


def build_kat_op(c, kat):
    """The coroutine for one KAT (operands as trivial/plain per the overload's types)."""
    args = []
    for t, v in zip(kat["types"], kat["args"]):
        if t.startswith("e"):
            args.append(I.FheUint.trivial(c, [v], _width(t)))
        else:
            args.append(int(v))
    return I.fhevm_op(c, kat["op"], *args)


def check_result(ck, kat, res):
    if kat["result_type"] == "ebool":
        got = int(ck.decrypt_bool(res)[0])
        return got == int(bool(kat["expect"]))
    return int(I.decrypt_bits(ck, res.bits)[0]) == kat["expect"] and res.width == _width(kat["result_type"])


@pytest.fixture(scope="module")
def kats():
    from conftest import load_kats
    return load_kats()


def test_fixture_sanity(kats):
    assert len(kats) == 2394                     # every overload, ebool .. euint256
    ops = {k["op"] for k in kats}
    assert ops == set(I.BINARY_OPS) | set(I.UNARY_OPS)
    for k in kats:
        assert k["source"].startswith("fhevmOperations") and ":" in k["source"]
        assert len(k["args"]) == len(k["types"])


def _py_semantics(op, types, args):
    w = max(_width(t) for t in types)
    m = (1 << w) - 1
    a = args[0]
    b = args[1] if len(args) > 1 else None
    sw = _width(types[0])
    if op in ("shl", "shr", "rotl", "rotr"):
        k = b % sw
        if op == "shl":
            return (a << k) & ((1 << sw) - 1)
        if op == "shr":
            return a >> k
        if op == "rotl":
            return ((a << k) | (a >> (sw - k))) & ((1 << sw) - 1)
        return ((a >> k) | (a << (sw - k))) & ((1 << sw) - 1)
    return {
        "add": lambda: (a + b) & m, "sub": lambda: (a - b) & m, "mul": lambda: (a * b) & m,
        "div": lambda: a // b if b else m, "rem": lambda: a % b if b else a,
        "and": lambda: a & b, "or": lambda: a | b, "xor": lambda: a ^ b,
        "eq": lambda: int(a == b), "ne": lambda: int(a != b), "ge": lambda: int(a >= b),
        "gt": lambda: int(a > b), "le": lambda: int(a <= b), "lt": lambda: int(a < b),
        "min": lambda: min(a, b), "max": lambda: max(a, b),
        "neg": lambda: (-a) & m, "not": lambda: (~a) & m,
    }[op]()


def test_fixture_matches_semantics(kats):
    """Our reading of the fhEVM semantics agrees with every expected value in the reference's KATs."""
    for k in kats:
        assert _py_semantics(k["op"], k["types"], k["args"]) == k["expect"], k


def test_all_kats_cleartext_lockstep(kats):
    eng = CleartextEngine(n=1)  # trivial ciphertexts: the mask width does not matter, memory does
    c = I.Circuit(eng)
    ck = ClearKey()
    results = c.run_many([build_kat_op(c, k) for k in kats])
    bad = [k for k, r in zip(kats, results) if not check_result(ck, k, r)]
    assert not bad, bad[:5]
    # one launch per level of the deepest circuit (not the sum over KATs)
    assert c.launches < 400, c.launches
    assert eng.min_margin >= (1 << 60), eng.min_margin   # >= 1/16 of the torus


@pytest.mark.parametrize("prefix", [True, False])
@pytest.mark.parametrize("w", [8, 16])
def test_add_sub_cmp_random(w, prefix):
    rng = np.random.default_rng(w + prefix)
    B = 64
    a = rng.integers(0, 1 << w, B, dtype=np.uint64)
    b = rng.integers(0, 1 << w, B, dtype=np.uint64)
    b[:8] = a[:8]                      # equal pairs for eq / ge boundaries
    eng = CleartextEngine()
    c = I.Circuit(eng)
    ck = ClearKey()
    A, Bv = I.FheUint.trivial(c, a, w), I.FheUint.trivial(c, b, w)
    s, _ = c.run(I.g_add(c, A.bits, Bv.bits, prefix=prefix))
    d, ge = c.run(I.g_add(c, A.bits, I.NOT(Bv.bits), True, want_carry=True, prefix=prefix))
    m = np.uint64((1 << w) - 1)
    np.testing.assert_array_equal(I.decrypt_bits(ck, s), (a + b) & m)
    np.testing.assert_array_equal(I.decrypt_bits(ck, d), (a - b) & m)
    np.testing.assert_array_equal(ck.decrypt_bool(ge), a >= b)
    _, ge2 = c.run(I.g_add(c, A.bits, I.NOT(Bv.bits), True, want_sum=False, want_carry=True, prefix=prefix))
    np.testing.assert_array_equal(ck.decrypt_bool(ge2), a >= b)
    eq = c.run(I.g_eq(c, A.bits, Bv.bits))
    np.testing.assert_array_equal(ck.decrypt_bool(eq), a == b)
    assert eng.min_margin >= (1 << 60)


def test_mul_divrem_random():
    rng = np.random.default_rng(7)
    w, B = 16, 32
    a = rng.integers(0, 1 << w, B, dtype=np.uint64)
    b = rng.integers(0, 1 << w, B, dtype=np.uint64)
    c = I.Circuit(CleartextEngine())
    ck = ClearKey()
    A, Bv = I.FheUint.trivial(c, a, w), I.FheUint.trivial(c, b, w)
    p = c.run(I.g_mul(c, A.bits, Bv.bits))
    np.testing.assert_array_equal(I.decrypt_bits(ck, p), (a * b) & np.uint64(0xFFFF))
    for d in (1, 3, 255, 256, 40000, 0):
        q, r = c.run(I.g_div_rem_scalar(c, A.bits, d))
        if d:
            np.testing.assert_array_equal(I.decrypt_bits(ck, q), a // np.uint64(d))
            np.testing.assert_array_equal(I.decrypt_bits(ck, r), a % np.uint64(d))
        else:
            assert (I.decrypt_bits(ck, q) == 0xFFFF).all()
            np.testing.assert_array_equal(I.decrypt_bits(ck, r), a)


def test_encrypted_shift_amounts_wrap():
    c = I.Circuit(CleartextEngine())
    ck = ClearKey()
    vals = np.array([0x1234, 0x8001, 0xFFFF, 0x0F0F], dtype=np.uint64)
    A = I.FheUint.trivial(c, vals, 16)
    for amt in (0, 1, 5, 15, 16, 17, 200):
        K = I.FheUint.trivial(c, [amt] * 4, 8)
        for kind in ("shl", "shr", "rotl", "rotr"):
            enc = c.run(I.fhevm_op(c, kind, A, K))
            clr = c.run(I.fhevm_op(c, kind, A, amt))
            want = [_py_semantics(kind, ["euint16", "uint8"], [int(v), amt]) for v in vals]
            np.testing.assert_array_equal(I.decrypt_bits(ck, enc.bits), want)
            np.testing.assert_array_equal(I.decrypt_bits(ck, clr.bits), want)


def test_operator_errors():
    c = I.Circuit(CleartextEngine())
    A = I.FheUint.trivial(c, [1], 8)
    with pytest.raises(ValueError):
        c.run(I.fhevm_op(c, "pow", A, 2))
    with pytest.raises(ValueError):
        c.run(I.fhevm_op(c, "add", 1, 2))
    with pytest.raises(ValueError):
        c.run(I.fhevm_op(c, "div", A, A))


# ---- the device-resident circuit (Circuit(device=...)): the same circuits on torch int64 tensors ---------------
class CleartextTorchEngine(CleartextEngine):
    """pbs_device of the cleartext double on torch CPU tensors (the device path's array code on CPU)."""

    def pbs_device(self, d_in, d_lut):
        import torch
        out = self.pbs(d_in.numpy().view(np.uint64), d_lut)
        return torch.from_numpy(out.view(np.int64))


def test_device_resident_circuit_matches_host(kats):
    """Every operator of a KAT sample and the C5 max tree give the same bits on torch tensors as on numpy
    arrays, through the same number of launches."""
    import torch
    for kat in kats[::25]:
        res = []
        for dev in (None, "cpu"):
            c = I.Circuit(CleartextTorchEngine(), device=dev)
            out = c.run(build_kat_op(c, kat))
            bits = out.bits if isinstance(out, I.FheUint) else out
            if isinstance(bits, torch.Tensor):
                bits = bits.numpy().view(np.uint64)
            res.append((bits.copy(), c.launches, c.pbs_count))
        assert np.array_equal(res[0][0], res[1][0]) and res[0][1:] == res[1][1:], kat
        assert check_result(ClearKey(), kat, I.FheUint(None, res[1][0]) if res[1][0].ndim == 3 else res[1][0])
    from tfhe_amd.auction import max_tree
    v = np.random.default_rng(11).integers(0, 2**32, 100, dtype=np.uint64)
    c = I.Circuit(CleartextTorchEngine(), device="cpu")
    mx, idx = max_tree(c, I.FheUint.trivial(c, v, 32))
    ck = ClearKey()
    assert isinstance(mx.bits, torch.Tensor)
    assert (int(mx.decrypt(ck)[0]), int(idx.decrypt(ck)[0])) == (int(v.max()), int(np.argmax(v)))
