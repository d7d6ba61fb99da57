"""CPU check of the arithmetic behind the matrix-core keyswitch (tfhe_amd/csrc/ks_mfma.hip):
balanced byte recoding of KSK words and the eight-plane int8 product, restated in numpy and
compared with the u64 wrapping product (the oracle's or_keyswitch rule) on random and edge words."""
import numpy as np

M64 = (1 << 64) - 1


def recode(k):
    """ksk_planes_kernel: bytes + carry, s_t = v - 256 if v >= 128, carry out of byte 7 dropped."""
    s, carry = [], 0
    for t in range(8):
        v = ((k >> (8 * t)) & 0xFF) + carry
        carry = 1 if v >= 128 else 0
        s.append(v - 256 if carry else v)
    return s


def test_recoding_identity_and_range():
    rng = np.random.default_rng(5)
    words = [0, 1, 127, 128, 255, 256, 2**63, M64, 0x8080808080808080, 0x7F7F7F7F7F7F7F7F] + \
        [int(x) for x in rng.integers(0, 2**64 - 1, 20000, dtype=np.uint64)]
    for k in words:
        s = recode(k)
        assert all(-128 <= v <= 127 for v in s)
        assert sum(v << (8 * t) for t, v in enumerate(s)) & M64 == k


def test_plane_product_equals_wrapping_product():
    """sum_k d_k KSK_k (mod 2^64) == sum_t 2^(8t) (sum_k d_k s_t,k), each plane sum exact in int32."""
    rng = np.random.default_rng(6)
    for K, dmax in ((8192, 2), (8192, 8)):  # P-GATE 2^2 x 8 and P-FHEVM 2^4 x 4, K = kN * levels
        d = rng.integers(-dmax, dmax + 1, K)
        ksk = [int(x) for x in rng.integers(0, 2**64 - 1, K, dtype=np.uint64)]
        ksk[:4] = [M64, 2**63, 0x8080808080808080, 0]
        S = np.array([recode(k) for k in ksk], dtype=np.int64)  # K x 8
        C = d @ S                                                 # the eight int8 GEMM columns
        assert np.abs(C).max() < 2**31 and K * 128 * dmax < 2**31
        got = sum(int(c) << (8 * t) for t, c in enumerate(C)) & M64
        want = sum(int(dk) * kk for dk, kk in zip(d, ksk)) & M64
        assert got == want
