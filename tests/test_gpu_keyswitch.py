"""GPU parity of the matrix-core keyswitch (tfhe_amd/csrc/ks_mfma.hip) through the C ABI.

Bit-exact against the oracle (or_keyswitch) on ragged batches that cross the 256-ciphertext
workgroup tile and on edge inputs (0, 2^63, all ones, exact rounding ties of the closest-representable
step), and bit-identical to the VALU keyswitch kernel (TFHE_HIP_KS_VALU=1) on a full 4096 batch —
a size-independent check of every output word — at both parameter sets (P-GATE 2^2 x 8,
P-FHEVM 2^4 x 4).
"""
import os

import numpy as np
import pytest

import tfhe_amd

pytestmark = pytest.mark.gpu


def _edge_rows(big_dim, ks_prec_bits, rng):
    tie = 1 << (63 - ks_prec_bits)  # the dropped low bits at exactly one half: a rounding tie
    rows = [np.zeros(big_dim + 1, np.uint64), np.full(big_dim + 1, 2**64 - 1, np.uint64),
            np.full(big_dim + 1, 2**63, np.uint64)]
    r = rng.integers(0, 2**64 - 1, big_dim + 1, dtype=np.uint64)
    r &= np.uint64((2**64 - 1) ^ ((tie << 1) - 1))
    rows.append(r | np.uint64(tie))          # ties everywhere
    rows.append(r | np.uint64(tie - 1))      # just below the tie
    return np.stack(rows)


def _valu_engine(params, sk):
    os.environ["TFHE_HIP_KS_VALU"] = "1"
    try:
        eng = tfhe_amd.Engine(params, 0)
    finally:
        del os.environ["TFHE_HIP_KS_VALU"]
    eng.load_keys(sk)
    return eng


@pytest.mark.parametrize("B", [1, 255, 257, 300])
def test_mfma_keyswitch_ragged_vs_oracle(engine, oracle_mod, gate_params, oracle_keys, B):
    rng = np.random.default_rng(100 + B)
    big = rng.integers(0, 2**64 - 1, size=(B, 1025), dtype=np.uint64)
    if B >= 5:
        big[:5] = _edge_rows(1024, 16, rng)
    out = engine.keyswitch(big)
    for i in sorted({0, 1, 2, 3, 4, B // 2, B - 1} & set(range(B))):
        assert np.array_equal(out[i], oracle_mod.keyswitch(gate_params, oracle_keys, big[i])), i


def test_mfma_keyswitch_equals_valu_kernel_4096(engine, product_keys):
    ck, sk = product_keys
    rng = np.random.default_rng(7)
    big = rng.integers(0, 2**64 - 1, size=(4096, 1025), dtype=np.uint64)
    big[:5] = _edge_rows(1024, 16, rng)
    out = engine.keyswitch(big)
    with _valu_engine(ck.params, sk) as ref_eng:
        ref = ref_eng.keyswitch(big)
    assert np.array_equal(out, ref)


def test_mfma_keyswitch_fhevm(fhevm_engine, fhevm_keys, oracle_mod):
    ck, sk = fhevm_keys
    prm = oracle_mod.params(1)
    keys = oracle_mod.Keys(prm, 0x7F4E0001)
    rng = np.random.default_rng(8)
    big = rng.integers(0, 2**64 - 1, size=(517, 2049), dtype=np.uint64)
    big[:5] = _edge_rows(2048, 16, rng)
    out = fhevm_engine.keyswitch(big)
    for i in (0, 1, 2, 3, 4, 256, 516):
        assert np.array_equal(out[i], oracle_mod.keyswitch(prm, keys, big[i])), i
    with _valu_engine(ck.params, sk) as ref_eng:
        assert np.array_equal(out, ref_eng.keyswitch(big))
