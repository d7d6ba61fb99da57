"""FFT64 transform on CPU: the oracle restatement (oracle/fft_oracle.c) against its definition, the
exact torus product it approximates, and the product's host-side keygen.

The f64 FFT is tfhe-rs's own external-product arithmetic ("tfhe-rs uses an f64 FFT"); the
reference's exact wrapping product (ml/extensions/rust/src/computations.rs:50-54) is the arbiter of
its rounding error here.  Device parity (bit-exact against this oracle) is tests/test_gpu_fft.py.
"""
import math

import numpy as np
import pytest

from conftest import KEY_SEED

N, M = 1024, 512


# device order: slot d = L + 64 e holds frequency k = (L >> 3) + 8 (L & 7) + 64 e
_D = np.arange(M)
DEVICE_ORDER = (_D % 64 >> 3) + 8 * (_D % 8) + 64 * (_D // 64)


def _dft_definition(a):
    """z_j = (a_j + i a_{j+M}) zeta^j, Z_k = sum_j z_j e^{+2 pi i jk/M}, returned in device order."""
    zeta = np.exp(1j * np.pi * np.arange(M) / N)
    z = (a[:M] + 1j * a[M:]) * zeta
    return (np.fft.ifft(z) * M)[DEVICE_ORDER]  # numpy's ifft uses e^{+2 pi i jk/M} / M


def test_twiddles_match_libm(oracle_mod):
    for Mt in (512, 2048):
        for t in range(0, Mt, 7):
            c, s = oracle_mod.fft_twiddle(t, Mt)
            # libm's own argument 2*pi*t/M carries ~1 ulp of rounding: compare at 1.5e-15
            assert abs(c - math.cos(2 * math.pi * t / Mt)) < 1.5e-15
            assert abs(s - math.sin(2 * math.pi * t / Mt)) < 1.5e-15
    # exact symmetry points
    assert oracle_mod.fft_twiddle(0, 512) == (1.0, 0.0)
    assert oracle_mod.fft_twiddle(128, 512) == (0.0, 1.0)
    assert oracle_mod.fft_twiddle(256, 512) == (-1.0, 0.0)


def test_forward_matches_definition(oracle_mod):
    rng = np.random.default_rng(3)
    for a in (rng.integers(-64, 64, N).astype(np.float64),
              rng.integers(-2**62, 2**62, N).astype(np.float64)):
        Z = oracle_mod.fft_fwd(a)[0]
        ref = _dft_definition(a)
        assert np.max(np.abs(Z - ref)) <= 1e-12 * np.max(np.abs(ref)) + 1e-9


def test_inverse_roundtrip(oracle_mod):
    rng = np.random.default_rng(4)
    a = rng.integers(-2**40, 2**40, N).astype(np.float64)
    back = oracle_mod.fft_inv(oracle_mod.fft_fwd(a))[0] / M
    # 2^40-scale inputs: ~2^-50 relative (max 1.1e-3 over 20 seeds, rms 2.7e-4 with the merged twist)
    assert np.max(np.abs(back - a)) < 2e-3


def test_product_vs_exact_torus_schoolbook(oracle_mod):
    """digit polynomial (|d| <= 64) x uniform torus polynomial: FFT product rounded to the torus stays
    within 2^28 of the exact wrapping product (2^-36 of the torus)."""
    rng = np.random.default_rng(5)
    worst = 0
    for _ in range(4):
        d = rng.integers(-64, 65, N)
        b = rng.integers(0, 2**64, N, dtype=np.uint64)
        Fb = oracle_mod.fft_fwd(b.view(np.int64).astype(np.float64))[0] * 2.0**-9
        prod = oracle_mod.fft_inv(oracle_mod.fft_fwd(d.astype(np.float64))[0] * Fb)[0]
        got = np.array([oracle_mod.f64_to_torus(x) for x in prod], dtype=np.uint64)
        ref = oracle_mod.poly_mul_torus_schoolbook(d, b)
        err = np.abs((got - ref).view(np.int64).astype(np.float64))
        worst = max(worst, float(err.max()))
    assert worst < 2.0**28, f"FFT product error 2^{math.log2(worst):.1f}"


def test_f64_to_torus_rounding(oracle_mod):
    f = oracle_mod.f64_to_torus
    assert f(2.5) == 2 and f(3.5) == 4 and f(-2.5) == (1 << 64) - 2  # ties to even
    assert f(-1.0) == (1 << 64) - 1 and f(0.49) == 0 and f(-0.0) == 0
    assert f(2.0**64 + 2.0**20) == 2**20
    assert f(-(2.0**70) + 2.0**30) == 2**30
    assert f(2.0**63) == 2**63 and f(-(2.0**63)) == 2**63


def test_device_accumulator_increment(oracle_mod):
    """or_f64_to_torus_dev (the device's rint-free update, fft512.h torus_acc_add[_wide]): equal to rint(x) mod 2^64
    for every |x| >= 2^32 and every x >= 0, and off by at most one for tiny negative x (x + 2^32 rounded once before
    the integer rounding); the two bit-pattern words of the device form restated in Python agree with it."""
    import struct
    f, g = oracle_mod.f64_to_torus_dev, oracle_mod.f64_to_torus
    rng = np.random.default_rng(0xACC)
    xs = np.concatenate([rng.standard_normal(400) * 2.0 ** rng.integers(0, 106, 400),
                         np.array([0.5, 1.5, 2.5, -0.5, -1.5, 2.0 ** 32 - 0.5, -(2.0 ** 32) + 0.5, 2.0 ** 63, -(2.0 ** 63),
                                   2.0 ** 83 - 2.0 ** 31, -(2.0 ** 81.5), 2.0 ** 105, -(2.0 ** 105) + 2.0 ** 60])])
    for x in xs.tolist():
        if abs(x) >= 2.0 ** 32 or x >= 0:
            assert f(x) == g(x), x
        else:
            assert (f(x) - g(x)) % 2 ** 64 in (0, 1, 2 ** 64 - 1), x

        def bits(d):
            return struct.unpack("<Q", struct.pack("<d", d))[0]
        h = math.floor(x * 2.0 ** -32)
        l = float(np.float64(x) - np.float64(h) * 2.0 ** 32)   # h 2^32 is exact: one rounding, as the fma
        hh = math.floor(h * 2.0 ** -32)
        hm = float(h - hh * 2 ** 32)
        dev = ((bits(hm + (1.5 * 2.0 ** 52 - 1127219200.0)) << 32) + bits(l + 2.0 ** 52)) % 2 ** 64
        assert dev == f(x), x
    assert (f(-0.5 - 2.0 ** -30) - g(-0.5 - 2.0 ** -30)) % 2 ** 64 == 1   # the double-rounding case, restated


def test_scaled_accumulator_update_forms(oracle_mod):
    """Round 5 (FFT_Y32 / F1_Y32): the keys' spectra carry 2^-32, so the inverse returns y = x 2^-32 and the device
    updates from y (fft512.h torus_acc_add_y at N = 1024, torus_acc_add_wide_y at N = 2048).  Restated here in IEEE
    double steps (numpy float64, one rounding per operation): both forms give or_f64_to_torus_dev(x) bit for bit,
    the wide one for every |x| < 2^96 (P-FHEVM reaches ~2^91), the N = 1024 one for |x| < 2^83 (P-GATE: 2^81.6)."""
    import struct
    f = oracle_mod.f64_to_torus_dev
    f64 = np.float64

    def bits(d):
        return struct.unpack("<Q", struct.pack("<d", float(d)))[0]
    rng = np.random.default_rng(0x5CA1ED)
    xs = np.concatenate([rng.standard_normal(600) * 2.0 ** rng.integers(0, 96, 600),
                         rng.integers(-2 ** 62, 2 ** 62, 100).astype(np.float64) + 0.5,
                         np.array([0.0, -0.0, 0.5, -0.5, 1.5, -1.5, 2.0 ** 32 - 0.5, -(2.0 ** 32) + 0.5, 2.0 ** 52,
                                   -(2.0 ** 52) - 1.0, 2.0 ** 63, -(2.0 ** 63), 2.0 ** 64 - 2.0 ** 11, 2.0 ** 80 + 2.0 ** 31,
                                   -(2.0 ** 81.5), 2.0 ** 95, -(2.0 ** 95) + 2.0 ** 50, -0.5 - 2.0 ** -30])])
    acc = 0x0123456789ABCDEF
    for x in xs.tolist():
        y = f64(x) * f64(2.0 ** -32)                       # exact: what the scaled pipeline returns
        h = np.floor(y)
        lb = (y - h) + f64(2.0 ** 20)
        want = (acc + f(x)) % 2 ** 64
        hb = (h * f64(2.0 ** -32) - np.floor(h * f64(2.0 ** -32))) + f64(2.0 ** 20)   # fract(h 2^-32) + 2^20
        hi = ((bits(hb) & 0xFFFFFFFF) - 0x41300000) % 2 ** 32
        assert (acc + (hi << 32) + bits(lb)) % 2 ** 64 == want, x
        if abs(x) < 2.0 ** 83:
            hb1 = h + f64(1.5 * 2.0 ** 52 - 1093664768.0)
            assert (acc + ((bits(hb1) & 0xFFFFFFFF) << 32) + bits(lb)) % 2 ** 64 == want, x


def test_negated_digit_form():
    """F1_NEGDIG (pbs_fft2k.hip dig23_neg): (int)(255 - h) >> 9 == -dig23(h) for the high word h of the rotated
    difference (checked on the device build for all 2^32 words; here on every 2^20-th word, the ties and the wrap)."""
    h = np.concatenate([np.arange(0, 2 ** 32, 2 ** 12, dtype=np.uint64),
                        np.arange(2 ** 31 - 1024, 2 ** 31 + 1024, dtype=np.uint64),
                        np.arange(0, 1024, dtype=np.uint64), np.arange(2 ** 32 - 1024, 2 ** 32, dtype=np.uint64),
                        (np.arange(0, 2 ** 23, dtype=np.uint64) << np.uint64(9)) + np.uint64(256)]) % 2 ** 32
    h = h.astype(np.uint32)
    dig = ((h + np.uint32(256 + (0x3FFFFF << 9))) >> np.uint32(9)).astype(np.int64) - 0x3FFFFF
    neg = (np.uint32(255) - h).view(np.int32) >> 9
    assert np.array_equal(neg.astype(np.int64), -dig)


def test_product_keygen_matches_oracle(oracle_mod):
    """tfhe_hip_keygen on the FFT64 preset: native-torus BSK bit-identical to or_keygen (host code)."""
    import tfhe_amd
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT)
    assert p.transform == tfhe_amd.TRANSFORM_FFT64 and p.N == 1024 and p.n == 630
    ck, sk = tfhe_amd.gen_keys(p, KEY_SEED)
    ok = oracle_mod.Keys(oracle_mod.params(2), KEY_SEED)
    assert np.array_equal(sk.bsk, ok.bsk)
    assert np.array_equal(sk.ksk, ok.ksk)
    # same secret keys as the NTT preset; the BSKs differ (torus vs Z_p GGSW)
    ok0 = oracle_mod.Keys(oracle_mod.params(0), KEY_SEED, with_bsk=False, with_ksk=False)
    assert np.array_equal(ok.lwe_key, ok0.lwe_key) and np.array_equal(ok.glwe_key, ok0.glwe_key)


@pytest.fixture(scope="module")
def fft_keys(oracle_mod):
    return oracle_mod.Keys(oracle_mod.params(2), KEY_SEED)


def test_oracle_pbs_decrypts(oracle_mod, fft_keys):
    prm = oracle_mod.params(2)
    rng = np.random.default_rng(6)
    bits = rng.integers(0, 2, 32)
    cts = fft_keys.encrypt([oracle_mod.encode_bit(int(b)) for b in bits], seed=0xC0FFEE21)
    out = oracle_mod.pbs_batch(prm, fft_keys, cts, oracle_mod.lut_constant(N, oracle_mod.MU)[None])
    ph = fft_keys.phase(out)
    assert [oracle_mod.decode_bit(int(x)) for x in ph] == [int(b) for b in bits]
    err = [((int(x) - oracle_mod.encode_bit(int(b))) + 2**63) % 2**64 - 2**63 for x, b in zip(ph, bits)]
    assert max(abs(e) for e in err) < 2**60  # 1/16 of the torus: inside the 1/8 gate margin


@pytest.mark.parametrize("lanes", [4, 8])
def test_simd_port_equals_scalar_restatement(oracle_mod, fft_keys, monkeypatch, lanes):
    """oracle/fft_batch.c (the CPU port bench.py times) runs fft_oracle.c's operations on 4 (AVX2) or 8 (AVX-512F)
    ciphertexts per vector: every output word equals the scalar restatement's, over a ragged group, two LUTs by
    lut_index, skipped CMUXes (mask words that switch to 0) and the rotation's wrapped half (a >= N)."""
    if lanes == 4:
        monkeypatch.setenv("ORACLE_SIMD_LANES", "4")
    elif oracle_mod.simd_lanes() != 8:
        pytest.skip("no AVX-512F on this CPU")
    assert oracle_mod.simd_lanes() == lanes
    prm = oracle_mod.params(2)
    rng = np.random.default_rng(40 + lanes)
    B = lanes + 3
    cts = rng.integers(0, 2**64, (B, prm.n + 1), dtype=np.uint64)
    cts[1, : prm.n : 3] = 0
    cts[2, : prm.n : 2] = np.uint64(3 << 62)  # switches to a = 1536 >= N
    luts = np.stack([oracle_mod.lut_constant(N, oracle_mod.MU),
                     oracle_mod.lut_from_table(N, 8, [(5 * m + 2) % 8 for m in range(8)], (1 << 63) // 8)])
    idx = rng.integers(0, 2, B).astype(np.uint32)
    ref = oracle_mod.pbs_batch_fft(prm, fft_keys, cts, luts, idx)
    assert np.array_equal(oracle_mod.pbs_batch_fft_simd(prm, fft_keys, cts, luts, idx, threads=2), ref)
    with pytest.raises(ValueError):
        oracle_mod.pbs_batch_fft_simd(oracle_mod.params(0), fft_keys, cts, luts, idx)


@pytest.mark.parametrize("lanes", [4, 8])
def test_simd_port_equals_scalar_restatement_fhevm(oracle_mod, monkeypatch, lanes):
    """The same at P-FHEVM (N = 2048, 2^23 x 1, KS -> MS noise reduction -> BR -> SE): the 1024-point transforms, the
    one-chain MAC from zero and the grouped keyswitch on the lanes equal the scalar restatement word for word, with
    and without the noise reduction, over a ragged group and two LUTs."""
    if lanes == 4:
        monkeypatch.setenv("ORACLE_SIMD_LANES", "4")
    elif oracle_mod.simd_lanes() != 8:
        pytest.skip("no AVX-512F on this CPU")
    prm = oracle_mod.params(3)
    keys = oracle_mod.Keys(prm, KEY_SEED)
    rng = np.random.default_rng(50 + lanes)
    B = lanes + 2
    cts = rng.integers(0, 2**64, (B, prm.k * prm.N + 1), dtype=np.uint64)
    luts = np.stack([oracle_mod.lut_constant(prm.N, 1 << 59), oracle_mod.lut_constant(prm.N, 3 << 59)])
    idx = rng.integers(0, 2, B).astype(np.uint32)
    for ms in (True, False):
        ref = oracle_mod.pbs_batch_fft(prm, keys, cts, luts, idx, ms=ms)
        assert np.array_equal(oracle_mod.pbs_batch_fft_simd(prm, keys, cts, luts, idx, threads=2, ms=ms), ref)


def test_oracle_blind_rotate_lut_table(oracle_mod, fft_keys):
    """decrypt(BR(m)) == f(m) for every message of an 8-valued table (biometrics main.rs:65-77)."""
    prm = oracle_mod.params(2)
    delta = (1 << 63) // 8
    table = [(3 * m + 1) % 8 for m in range(8)]
    lut = oracle_mod.lut_from_table(N, 8, table, delta)
    msgs = [m * delta for m in range(8)]
    cts = fft_keys.encrypt(msgs, seed=0xC0FFEE22)
    for m in range(8):
        acc = oracle_mod.blind_rotate_fft(prm, fft_keys, cts[m], lut)
        big = oracle_mod.sample_extract_torus(prm, acc)
        ph = fft_keys.phase(big, fft_keys.glwe_key, N)[0]
        assert ((int(ph) + delta // 2) // delta) % 16 == table[m]


def test_device_decomposition_steps_equal_signed_decomposer(oracle_mod):
    """pbs_fft.hip decomposes least-significant level first with a running state
    (W = st + 63 + b, b = bit 13 of st below the top level): equal to the tfhe-rs SignedDecomposer rule
    for every 21-bit state (exhaustive, numpy), and to or_decompose on sampled torus values."""
    V = np.arange(1 << 21, dtype=np.int64)

    def sequential(st):
        out = []
        for _ in range(3):
            res = st & 127
            st = st >> 7
            carry = ((((res - 1) | st) & res) >> 6) & 1
            st = st + carry
            out.append(res - (carry << 7))
        return out

    def steps(st):
        out = []
        for q in range(3):
            b = (st >> 13) & 1 if q < 2 else np.zeros_like(st)
            W = st + 63 + b
            out.append((W & 127) - 63 - b)
            st = W >> 7
        return out

    assert all(np.array_equal(a, b) for a, b in zip(sequential(V), steps(V)))
    rng = np.random.default_rng(8)
    for x in list(rng.integers(0, 2**64, 3000, dtype=np.uint64)) + [0, 2**64 - 1, 2**63, 2**42, 2**42 - 1]:
        x = int(x)
        st = np.array([(((x >> 32) + 1024) % 2**32) >> 11], dtype=np.int64)  # the device's decomp_state
        lv = [int(v[0]) for v in steps(st)]  # least significant first
        assert lv[::-1] == oracle_mod.decompose(x, 7, 3)


def test_decomp_23x1_high_word_restatement(oracle_mod):
    """pbs_fft2k.hip (dig23) decomposes 2^23 x 1 from the high word alone: st = (hi + 2^8) >> 9,
    digit = ((st + 2^22 - 1) mod 2^23) - (2^22 - 1).  Equal to or_decompose on edge and random words."""
    rng = np.random.default_rng(23)
    his = [0, 1, 255, 256, 511, 512, 2**31, 2**32 - 1, 2**32 - 256, 2**32 - 257, 2**32 - 512, 2**30 + 2**9 - 1,
           2**30 + 2**8, (2**22) << 9, ((2**22) << 9) - 256, ((2**22) << 9) + 255, ((2**22 + 1) << 9) - 256]
    his += [int(v) for v in rng.integers(0, 2**32, 4000, dtype=np.uint64)]
    for hi in his:
        for lo in (0, 2**32 - 1, int(rng.integers(0, 2**32))):
            x = (hi << 32) | lo
            st = ((hi + 256) % 2**32) >> 9
            d = ((st + 0x3FFFFF) & 0x7FFFFF) - 0x3FFFFF
            assert [d] == oracle_mod.decompose(x, 23, 1), (hi, lo)


def _fast_f64_to_torus(x: float) -> int:
    """pbs_fft.hip's f64_to_torus (fft512.h), restated: rint, h = floor(t / 2^32), l = t - h 2^32, and the low
    word of h taken from the mantissa of h + 1.5 * 2^52 -- exact only while |h| < 2^51, i.e. |x| < 2^83."""
    import struct
    t = float(np.rint(x))
    h = math.floor(t * 2.0 ** -32)
    l = t - h * 2.0 ** 32
    hm = struct.unpack("<Q", struct.pack("<d", float(h) + 1.5 * 2.0 ** 52))[0] & 0xFFFFFFFF
    return (hm << 32) | int(l)


def test_pgate_inverse_output_bound_fast_torus_path(oracle_mod):
    """P-GATE's inverse-transform outputs stay inside the fast f64_to_torus range by linearity:
    |sum over (k+1)l = 6 rows of d (*) BSK| <= 6 * N * 2^6 * 2^63 = 2^81.58 < 2^83.  Adversarial case: every BSK
    coefficient -2^63, digits +-64 signed so one output coefficient reaches the bound exactly; the fast form
    equals the oracle's exact two-split form on every output."""
    bound = 6 * N * 64 * 2 ** 63
    assert math.log2(bound) < 81.6 and bound < 2 ** 83
    bsk_poly = np.full(N, -2.0 ** 63)
    K = oracle_mod.fft_fwd(bsk_poly)[0] / M          # or_bsk_to_fourier: x 2^-9
    for k_peak in (0, 511, N - 1):
        O = np.zeros(M, dtype=np.complex128)
        for r in range(6):
            d = np.where(np.arange(N) <= k_peak, 64.0, -64.0)   # coefficient k_peak sums every term with one sign
            D = oracle_mod.fft_fwd(d)[0]
            O = O + D * K
        x = oracle_mod.fft_inv(O)[0]
        assert np.max(np.abs(x)) < 2.0 ** 83
        assert abs(abs(x[k_peak]) - bound) <= 2.0 ** 40   # the peak coefficient reaches the linear bound
        for v in x[:: 37].tolist() + [x[k_peak]]:
            assert _fast_f64_to_torus(v) == oracle_mod.f64_to_torus(v)


# ---- N = 2048: the one-wave 1024-point transform (fft_oracle.c fft1k_*, fft1k.h / pbs_fft2k.hip) ---------------
N2, M2 = 2048, 1024
_L, _S = np.arange(M2) % 64, np.arange(M2) // 64
# device index L + 64 m1 holds frequency k = (L & 3) + 4 (L >> 4) + 16 ((L >> 2) & 3) + 64 m1
DEVICE_ORDER_1K = (_L & 3) + 4 * (_L >> 4) + 16 * ((_L >> 2) & 3) + 64 * _S


def _dft_definition_2k(a):
    zeta = np.exp(1j * np.pi * np.arange(M2) / N2)
    z = (a[:M2] + 1j * a[M2:]) * zeta
    return (np.fft.ifft(z) * M2)[DEVICE_ORDER_1K]


def test_fft1k_is_a_permutation_of_frequencies():
    assert np.array_equal(np.sort(DEVICE_ORDER_1K), np.arange(M2))


def test_fft2k_forward_matches_definition(oracle_mod):
    rng = np.random.default_rng(13)
    for a in (rng.integers(-2**22, 2**22, N2).astype(np.float64),
              rng.integers(-2**62, 2**62, N2).astype(np.float64)):
        Z = oracle_mod.fft_fwd(a)[0]
        ref = _dft_definition_2k(a)
        assert np.max(np.abs(Z - ref)) <= 1e-12 * np.max(np.abs(ref)) + 1e-9


def test_fft2k_inverse_roundtrip(oracle_mod):
    rng = np.random.default_rng(14)
    a = rng.integers(-2**40, 2**40, N2).astype(np.float64)
    back = oracle_mod.fft_inv(oracle_mod.fft_fwd(a))[0] / M2
    assert np.max(np.abs(back - a)) < 4e-3


def test_fft2k_product_vs_exact_torus_schoolbook(oracle_mod):
    """23-bit digits x uniform torus polynomial (the P-FHEVM external product): the transform's product rounded with
    the wide torus path stays within 2^42 of the exact wrapping product (measured 2^39.7; round 3's two-wave form:
    2^40.0)."""
    rng = np.random.default_rng(15)
    worst = 0
    for _ in range(2):
        d = rng.integers(-2**22, 2**22 + 1, N2)
        b = rng.integers(0, 2**64, N2, dtype=np.uint64)
        Fb = oracle_mod.fft_fwd(b.view(np.int64).astype(np.float64))[0] * 2.0**-10
        prod = oracle_mod.fft_inv(oracle_mod.fft_fwd(d.astype(np.float64))[0] * Fb)[0]
        got = np.array([oracle_mod.f64_to_torus(x) for x in prod], dtype=np.uint64)
        ref = oracle_mod.poly_mul_torus_schoolbook(d, b)
        err = np.abs((got - ref).view(np.int64).astype(np.float64))
        worst = max(worst, float(err.max()))
    assert worst < 2.0**42, f"product error 2^{math.log2(worst):.1f}"
