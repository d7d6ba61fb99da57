"""fhEVM operator KATs replayed on the MI355X (message-level parity).

Every KAT of the reference's tests/fhevm-suite/e2e/test/fhevmOperations*.ts -- all 2,394 overloads,
ebool and euint8 .. euint256 (fixture tests/golden/fhevm_kats.json) -- is encrypted under the
P-GATE key, evaluated by tfhe_amd.integer through the GPU gate bootstrap (libtfhe_hip.so) — all
KATs in lockstep, one PBS launch per circuit level — and decrypted.  Expected values are the
reference's own `expect(res).to.equal(...)` constants.
"""
import json
import os

import numpy as np
import pytest

from tfhe_amd import integer as I

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "fhevm_kats.json")


def _width(t):
    return 1 if t == "ebool" else int(t.lstrip("e").replace("uint", ""))


@pytest.mark.parametrize("transform", ["ntt", "fft64"])
def test_fhevm_kats_gpu(request, transform):
    engine = request.getfixturevalue("engine" if transform == "ntt" else "gate_fft_engine")
    ck, _ = request.getfixturevalue("product_keys" if transform == "ntt" else "gate_fft_keys")
    from conftest import load_kats
    # all 2,394 on the FFT64 engine (the default); the NTT engine replays the ebool .. euint64 overloads
    # (1,464: the euint128 multipliers alone are ~2.3M PBS, ~75 s at that engine's rate)
    kats = load_kats() if transform == "fft64" else load_kats(max_width=64)
    assert len(kats) == (2394 if transform == "fft64" else 1464)
    c = I.Circuit(engine)
    ops, stream = [], 0
    for k in kats:
        args = []
        for t, v in zip(k["types"], k["args"]):
            if t.startswith("e"):
                w = _width(t)
                args.append(I.FheUint.encrypt(c, ck, [v], w, seed=0xF4E7, stream0=stream))
                stream += w
            else:
                args.append(int(v))
        ops.append(I.fhevm_op(c, k["op"], *args))
    results = c.run_many(ops)
    bad = []
    for k, r in zip(kats, results):
        if k["result_type"] == "ebool":
            got = int(ck.decrypt_bool(r)[0])
            ok = got == int(bool(k["expect"]))
        else:
            got = int(I.decrypt_bits(ck, r.bits)[0])
            ok = got == k["expect"] and r.width == _width(k["result_type"])
        if not ok:
            bad.append((k["source"], k["op"], k["types"], k["args"], k["expect"], got))
    assert not bad, f"{len(bad)} KATs failed, first: {bad[:5]}"
    assert c.launches <= 40, c.launches


@pytest.mark.parametrize("w", [8, 32])
def test_integer_batch_random_gpu(engine, product_keys, w):
    """A batch large enough to take the ripple (throughput) adders; compared with numpy."""
    ck, _ = product_keys
    rng = np.random.default_rng(w)
    B = 256 if w == 8 else 64
    a = rng.integers(0, 1 << w, B, dtype=np.uint64)
    b = rng.integers(0, 1 << w, B, dtype=np.uint64)
    b[:4] = a[:4]
    c = I.Circuit(engine, capacity=64)           # force the ripple path
    A = I.FheUint.encrypt(c, ck, a, w, seed=11, stream0=0)
    Bv = I.FheUint.encrypt(c, ck, b, w, seed=11, stream0=B * w)
    add, sub, lt, mx = c.run_many([I.fhevm_op(c, "add", A, Bv), I.fhevm_op(c, "sub", A, Bv),
                                   I.fhevm_op(c, "lt", A, Bv), I.fhevm_op(c, "max", A, Bv)])
    m = np.uint64((1 << w) - 1)
    np.testing.assert_array_equal(I.decrypt_bits(ck, add.bits), (a + b) & m)
    np.testing.assert_array_equal(I.decrypt_bits(ck, sub.bits), (a - b) & m)
    np.testing.assert_array_equal(ck.decrypt_bool(lt), a < b)
    np.testing.assert_array_equal(I.decrypt_bits(ck, mx.bits), np.maximum(a, b))
