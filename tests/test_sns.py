"""Switch-and-squash / noise squashing (tfhe_amd/sns.py) on CPU: product key
generation and decryption against the oracle (oracle/sns_oracle.c), the oracle's Z_Q NTT against a
schoolbook product, and the oracle pipeline end to end at the full parameter set (keyswitch ->
modulus-switch noise reduction -> 128-bit bootstrap) decrypting every message with ~2^-63 noise."""
import numpy as np
import pytest

from conftest import KEY_SEED
from tfhe_amd import sns as S


def test_preset():
    sp = S.SnsParams.preset(S.SNS_PRESET_FHEVM)
    assert (sp.n, sp.k, sp.N, sp.base_log, sp.level) == (918, 2, 2048, 24, 3)


def test_keygen_and_phase_match_oracle(oracle_mod):
    sp = S.SnsParams.preset(0)
    osp = oracle_mod.sns_params(0)
    sp.n = osp.n = 12                              # key structure at a reduced input dimension
    key = np.random.default_rng(2).integers(0, 2, 12).astype(np.uint64)
    a = S.SquashedKey(sp, KEY_SEED, key)
    b = oracle_mod.SnsKeys(osp, KEY_SEED, key)
    assert np.array_equal(a.glwe_key, b.glwe_key) and np.array_equal(a.bsk, b.bsk)
    assert a.bsk.size == 12 * 9 * 3 * 2 * 2048
    cts = np.random.default_rng(3).integers(0, 2 ** 64 - 1, size=(3, 4097, 2), dtype=np.uint64)
    assert a.phase(cts) == oracle_mod.sns_phase(osp, b.glwe_key, cts)


@pytest.mark.parametrize("which", [0, 1])
def test_oracle_ntt_is_negacyclic_product(oracle_mod, which):
    N = 64
    p = [0xFFFFFFFF00000001, 0xFFFFFFFC00000001][which]
    rng = np.random.default_rng(which)
    x = rng.integers(0, 2 ** 40, N).astype(object)
    y = rng.integers(0, 2 ** 40, N).astype(object)
    want = [0] * N
    for i in range(N):
        for j in range(N):
            t = x[i] * y[j]
            if i + j < N:
                want[i + j] += t
            else:
                want[i + j - N] -= t
    X = oracle_mod.sns_ntt(which, np.array(x, dtype=np.uint64))
    Y = oracle_mod.sns_ntt(which, np.array(y, dtype=np.uint64))
    Z = np.array([(int(a) * int(b)) % p for a, b in zip(X, Y)], dtype=np.uint64)
    got = oracle_mod.sns_ntt(which, Z, inverse=True)
    assert [int(v) for v in got] == [w % p for w in want]


def test_oracle_squash_end_to_end(oracle_mod):
    prm = oracle_mod.params(1)
    ok = oracle_mod.Keys(prm, KEY_SEED, with_bsk=False)
    osp = oracle_mod.sns_params(0)
    sk = oracle_mod.SnsKeys(osp, KEY_SEED, ok.lwe_key)
    msgs = np.array([0, 5, 10, 15], dtype=np.uint64)
    big = ok.encrypt(msgs * np.uint64((1 << 63) // 16), seed=0xC0FFEE70)
    small = np.stack([oracle_mod.keyswitch(prm, ok, c) for c in big])
    small, _ = oracle_mod.ms_reduce(prm, ok, small)
    out = oracle_mod.sns_squash(osp, sk, small, 16, threads=8)
    ph = oracle_mod.sns_phase(osp, sk.glwe_key, out)
    delta = 1 << 123
    assert [((v + delta // 2) // delta) % 16 for v in ph] == [int(m) for m in msgs]
    noise = [((v - int(m) * delta + (1 << 127)) % (1 << 128)) - (1 << 127) for v, m in zip(ph, msgs)]
    assert max(abs(e) for e in noise) < 2 ** 70      # squashed: ~2^65 of the 2^128 torus


def test_key_rounding(oracle_mod):
    """or_sns_bsk_round (the device's load-time rounding): every coefficient becomes the multiple of
    2^16 nearest to its centred value mod Q, so a rounded key is 2^16 x a 112-bit integer (seven
    balanced 16-bit limbs) and moves each coefficient by at most 2^15."""
    import ctypes
    osp = oracle_mod.sns_params(0)
    osp.n = 1
    keys = oracle_mod.SnsKeys(osp, KEY_SEED, np.array([1], dtype=np.uint64))
    out = np.zeros_like(keys.bsk)
    oracle_mod.lib().or_sns_bsk_round(ctypes.byref(osp), oracle_mod._p(keys.bsk), oracle_mod._p(out))
    p1, p2 = 0xFFFFFFFF00000001, 0xFFFFFFFC00000001
    Q = p1 * p2
    inv = pow(p1, -1, p2)

    def crt(r1, r2):
        return int(r1) + p1 * (((int(r2) - int(r1)) * inv) % p2)

    pairs = keys.bsk.reshape(-1, 2, 2048)
    rpairs = out.reshape(-1, 2, 2048)
    rng = np.random.default_rng(5)
    for pp in rng.integers(0, pairs.shape[0], 6):
        for t in rng.integers(0, 2048, 40):
            x = crt(pairs[pp, 0, t], pairs[pp, 1, t])
            y = crt(rpairs[pp, 0, t], rpairs[pp, 1, t])
            xc = x - Q if x > Q // 2 else x
            yc = y - Q if y > Q // 2 else y
            assert yc % 65536 == 0 and abs(yc - xc) <= 32768 and abs(yc // 65536) < 2 ** 111


def test_fft_limb_product_exactness(tmp_path):
    """tools/sns_fft_check.cpp runs the device's FFT stage functions (tfhe_amd/csrc/sns_fft.h) on the
    host: 9-term digit x limb products at N = 2048 with uniform and extreme-magnitude random operands
    land within 0.07 of the exact integers (rint() exact with margin), and the adversarial all-maximum
    operand (|value| = 2^52.2, no f64 headroom) is reported as the one inexact case."""
    import subprocess
    root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    exe = tmp_path / "sns_fft_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", f"{root}/tfhe_amd/csrc", f"{root}/tools/sns_fft_check.cpp",
                    "-o", str(exe)], check=True)
    for form in ("s", "w"):  # the 256-thread stage form (inverse, key conversion) and the one-wave form (step 1)
        out = subprocess.run([str(exe), "6", form], capture_output=True, text=True).stdout
        assert "stage form vs wave form spectra: max |diff| = 0.000e+00" in out
        errs = [(int(l.split()[3].rstrip(":")), float(l.split("=")[1].split(",")[0])) for l in out.splitlines()
                if l.startswith("trial")]
        assert len(errs) == 6
        assert all(e < 0.07 for mode, e in errs if mode != 2)
