"""Radix integers (tfhe_amd/radix.py) on the MI355X at the production fhEVM parameters: every
reference fhEVM operator KAT (all 2,394: ebool .. euint256, div/rem included), encrypted under the
P-FHEVM key, evaluated in lockstep (one multi-LUT PBS launch per circuit level) and decrypted."""
import json
import os

import numpy as np
import pytest

from tfhe_amd import radix as R
from conftest import load_kats
from test_radix import _w, supported

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("transform", ["ntt", "fft64"])
def test_radix_kats_gpu(request, transform):
    fhevm_engine = request.getfixturevalue("fhevm_engine" if transform == "ntt" else "fhevm_fft_engine")
    ck, _ = request.getfixturevalue("fhevm_keys" if transform == "ntt" else "fhevm_fft_keys")
    kats = [k for k in (load_kats() if transform == "fft64" else load_kats(max_width=64)) if supported(k)]
    assert len(kats) == (2394 if transform == "fft64" else 1464)
    c = R.RadixCircuit(fhevm_engine)
    ops, stream = [], 0
    for k in kats:
        args = []
        for t, v in zip(k["types"], k["args"]):
            if t.startswith("e"):
                w = _w(t)
                args.append(R.RadixUint.encrypt(c, ck, [v], w, seed=0x5AD1, stream0=stream))
                stream += w // 2
            else:
                args.append(int(v))
        ops.append(R.fhevm_op(c, k["op"], *args))
    res = c.run_many(ops)
    bad = []
    for k, r in zip(kats, res):
        if k["result_type"] == "ebool":
            got = int(ck.decrypt(r, R.SPACE)[0])
            ok = got == int(bool(k["expect"]))
        else:
            got = int(r.decrypt(ck)[0])
            ok = got == k["expect"]
        if not ok:
            bad.append((k["source"], k["op"], k["types"], k["args"], k["expect"], got))
    assert not bad, f"{len(bad)} of {len(kats)} failed: {bad[:5]}"
    assert c.launches <= 40


def test_radix_batch_gpu(fhevm_engine, fhevm_keys):
    ck, _ = fhevm_keys
    rng = np.random.default_rng(32)
    B, w = 256, 32
    a = rng.integers(0, 1 << w, B, dtype=np.uint64)
    b = rng.integers(0, 1 << w, B, dtype=np.uint64)
    c = R.RadixCircuit(fhevm_engine)
    A = R.RadixUint.encrypt(c, ck, a, w, seed=1, stream0=0)
    Bv = R.RadixUint.encrypt(c, ck, b, w, seed=1, stream0=B * 16)
    add, lt, mx = c.run_many([R.fhevm_op(c, "add", A, Bv), R.fhevm_op(c, "lt", A, Bv), R.fhevm_op(c, "max", A, Bv)])
    m = np.uint64((1 << w) - 1)
    np.testing.assert_array_equal(add.decrypt(ck), (a + b) & m)
    np.testing.assert_array_equal(ck.decrypt(lt, R.SPACE).astype(bool), a < b)
    np.testing.assert_array_equal(mx.decrypt(ck), np.maximum(a, b))


def test_radix_div_rem_gpu(fhevm_engine, fhevm_keys):
    """division / remainder by plaintext divisors (multiply-high, power-of-two and d = 0 paths)."""
    ck, _ = fhevm_keys
    rng = np.random.default_rng(77)
    B, w = 64, 32
    a = rng.integers(0, 1 << w, B, dtype=np.uint64)
    a[:2] = [0, (1 << w) - 1]
    c = R.RadixCircuit(fhevm_engine)
    A = R.RadixUint.encrypt(c, ck, a, w, seed=3, stream0=0)
    cases = [("div", 7), ("rem", 1000), ("div", 32), ("rem", 32), ("rem", 550954323), ("div", 0)]
    res = c.run_many([R.fhevm_op(c, op, A, d) for op, d in cases])
    for (op, d), r in zip(cases, res):
        if d == 0:
            want = np.full_like(a, (1 << w) - 1)
        else:
            want = a // np.uint64(d) if op == "div" else a % np.uint64(d)
        np.testing.assert_array_equal(r.decrypt(ck), want, err_msg=f"{op} {d}")
