"""Generate the FFT64 golden fixtures from the CPU oracle (run from the repo root):

    python tests/golden/make_golden_fft64.py

fft64_gate.npz (P-GATE, preset 2) and fft64_fhevm.npz (P-FHEVM, preset 3): inputs, blind-rotation accumulators
and full-PBS outputs of oracle/fft_oracle.c -- the FFT64 operation order the device kernels reproduce bit for
bit.  They exist so that a change of that order (kernel and oracle edited in lockstep) shows up as a fixture
diff: tests/test_oracle.py checks the oracle against them, tests/test_gpu_exact.py the device.  Keys are not
stored, only their seed (conftest.KEY_SEED).  Their distance to exact arithmetic is tests/test_exact.py's and
tests/test_gpu_exact.py's business (oracle/exact_oracle.c).  Ciphertext-level parity with tfhe-rs remains "parity unpinned" (oracle/tfhe_oracle.h).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

KEY_SEED = 0x7F4E0001
OUT = os.path.dirname(os.path.abspath(__file__))


def boundary_masks(n: int, N: int, rng) -> np.ndarray:
    """mask words on the modulus-switch rounding boundaries: odd multiples of 2^64 / 4N, minus 0 or 1"""
    half = np.uint64(1 << (63 - (2 * N).bit_length() + 1))
    t = rng.integers(0, 2 * N, n).astype(np.uint64)
    return (np.uint64(2) * t + np.uint64(1)) * half - rng.integers(0, 2, n).astype(np.uint64)


def gate():
    prm = O.params(2)
    keys = O.Keys(prm, KEY_SEED)
    rng = np.random.default_rng(0xF640)
    N = prm.N
    bits = [1, 0, 1, 0]
    cts = keys.encrypt([O.encode_bit(b) for b in bits], seed=0xC0FFEEF6)
    cts[3, :prm.n] = boundary_masks(prm.n, N, rng)
    luts = np.stack([O.lut_constant(N, O.MU), O.lut_from_table(N, 8, [(5 * m + 2) % 8 for m in range(8)],
                                                               (1 << 63) // 8)])
    idx = np.array([0, 1, 1, 0], dtype=np.uint32)
    acc = np.stack([O.blind_rotate_fft(prm, keys, cts[i], luts[idx[i]]) for i in range(4)])
    out = O.pbs_batch_fft(prm, keys, cts, luts, idx)
    np.savez(os.path.join(OUT, "fft64_gate.npz"), key_seed=np.uint64(KEY_SEED), preset=np.uint32(2), lwe_in=cts,
             luts=luts, lut_index=idx, acc=acc, lwe_out=out)


def fhevm():
    prm = O.params(3)
    keys = O.Keys(prm, KEY_SEED)
    N, mm = prm.N, 16
    delta = (1 << 63) // mm
    cts = keys.encrypt([m * delta for m in (0, 5, 11)], seed=0xC0FFEEF7)   # big-key inputs (KS -> PBS order)
    luts = np.stack([O.lut_from_table(N, mm, [(3 * m + 1) % mm for m in range(mm)], delta),
                     O.lut_from_table(N, mm, [(m * m) % mm for m in range(mm)], delta)])
    idx = np.array([0, 1, 0], dtype=np.uint32)
    small = np.stack([O.keyswitch(prm, keys, c) for c in cts])            # blind-rotation inputs (no MS reduction)
    acc = np.stack([O.blind_rotate_fft(prm, keys, small[i], luts[idx[i]]) for i in range(3)])
    out = O.pbs_batch_fft(prm, keys, cts, luts, idx)                      # KS -> MS reduction -> BR -> SE
    np.savez(os.path.join(OUT, "fft64_fhevm.npz"), key_seed=np.uint64(KEY_SEED), preset=np.uint32(3), lwe_in=cts,
             small=small, luts=luts, lut_index=idx, acc=acc, lwe_out=out)


if __name__ == "__main__":
    gate()
    fhevm()
    print("FFT64 golden fixtures written to", OUT)
