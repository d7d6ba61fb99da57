"""Host-side checks of the product library without a GPU: the C-ABI .so loads and exports every
symbol include/tfhe_hip.h declares; client-side key material (keygen / encrypt / LUT builders in
libtfhe_hip.so) is bit-identical to the oracle; device entry points fail cleanly (no abort)."""
import os
import re

import numpy as np
import pytest

from conftest import KEY_SEED, ROOT

import tfhe_amd


def header_functions():
    src = open(os.path.join(ROOT, "include", "tfhe_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tfhe_hip_\w+)\s*\(", src)))


def test_abi_exports_every_declared_symbol():
    L = tfhe_amd.lib()
    declared = header_functions()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(L, name), f"libtfhe_hip.so does not export {name}"
    assert sorted(tfhe_amd.ABI_SYMBOLS) == declared


def test_presets():
    g = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE)
    assert (g.n, g.k, g.N, g.pbs_base_log, g.pbs_level, g.ks_base_log, g.ks_level, g.order) == (630, 1, 1024, 7, 3, 2, 8, 0)
    f = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM)
    assert (f.n, f.k, f.N, f.pbs_base_log, f.pbs_level, f.ks_base_log, f.ks_level, f.order) == (918, 1, 2048, 23, 1, 4, 4, 1)
    L = tfhe_amd.lib()
    import ctypes
    assert L.tfhe_hip_bsk_len(ctypes.byref(g)) == 630 * 6 * 2 * 1024
    assert L.tfhe_hip_ksk_len(ctypes.byref(g)) == 1024 * 8 * 631
    with pytest.raises(tfhe_amd.TfheError):
        tfhe_amd.Params.preset(7)


def test_keygen_matches_oracle(product_keys, oracle_keys):
    ck, sk = product_keys
    assert np.array_equal(ck.lwe_key, oracle_keys.lwe_key)
    assert np.array_equal(ck.glwe_key, oracle_keys.glwe_key)
    assert np.array_equal(sk.bsk, oracle_keys.bsk)
    assert np.array_equal(sk.ksk, oracle_keys.ksk)
    assert int(sk.bsk.max()) < 0xFFFFFFFF00000001  # canonical Z_p


def test_keygen_and_encrypt_match_oracle_fhevm(oracle_mod):
    """P-FHEVM (N=2048, KS->PBS): keys, encryptions under the big (GLWE) key, LUTs."""
    prm = oracle_mod.params(1)
    ok = oracle_mod.Keys(prm, KEY_SEED)
    ck, sk = tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM), KEY_SEED)
    assert np.array_equal(ck.lwe_key, ok.lwe_key) and np.array_equal(ck.glwe_key, ok.glwe_key)
    assert np.array_equal(sk.bsk, ok.bsk) and np.array_equal(sk.ksk, ok.ksk)
    assert sk.ms_zeros.shape == (1449, 919) and np.array_equal(sk.ms_zeros, ok.ms_zeros)
    zph = ok.phase(sk.ms_zeros, ok.lwe_key, prm.n).view(np.int64)
    assert np.abs(zph).max() < 2 ** 50                       # encryptions of zero under the small key
    msgs = (np.arange(16, dtype=np.uint64) * np.uint64((1 << 63) // 16))
    a = ck.encrypt_torus(msgs, seed=0xC0FFEE03)
    assert a.shape == (16, 2049)
    assert np.array_equal(a, ok.encrypt(msgs, seed=0xC0FFEE03))
    assert np.array_equal(ck.decrypt(a, 16), np.arange(16))
    tab = [(m * m + 3) % 16 for m in range(16)]
    assert np.array_equal(tfhe_amd.lut_from_table(2048, 16, tab, (1 << 63) // 16),
                          oracle_mod.lut_from_table(2048, 16, tab, (1 << 63) // 16))


def test_encrypt_phase_matches_oracle(product_keys, oracle_keys):
    ck, _ = product_keys
    msgs = np.array([1 << 61, (1 << 64) - (1 << 61), 0, 12345], dtype=np.uint64)
    a = ck.encrypt_torus(msgs, seed=0xC0FFEE02, stream0=5)
    b = oracle_keys.encrypt(msgs, seed=0xC0FFEE02, stream0=5)
    assert np.array_equal(a, b)
    assert np.array_equal(ck.phase(a), oracle_keys.phase(b))
    err = (ck.phase(a) - msgs).astype(np.int64)
    assert np.abs(err).max() < 2**56


def test_lut_builders_match_oracle(oracle_mod):
    O = oracle_mod
    assert np.array_equal(tfhe_amd.lut_constant(1024, 1 << 61), O.lut_constant(1024, 1 << 61))
    for mm in (2, 4, 8, 16):
        tab = [(3 * m + 1) % mm for m in range(mm)]
        assert np.array_equal(tfhe_amd.lut_from_table(1024, mm, tab, (1 << 63) // mm),
                              O.lut_from_table(1024, mm, tab, (1 << 63) // mm))


def test_bad_arguments_fail_cleanly():
    with pytest.raises(tfhe_amd.TfheError) as e:
        tfhe_amd.lut_from_table(1024, 3, [0, 1, 2], 1)
    assert e.value.code == -1


def test_engine_without_gpu_raises_not_aborts():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present: covered by the gpu tests")
    except ImportError:
        pass
    with pytest.raises(tfhe_amd.TfheError):
        tfhe_amd.Engine(tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE), 0)


def test_unsupported_params_refused_on_device_build():
    # a parameter set without device kernels must be refused loudly (EUNSUPPORTED), never computed
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM)
    p.ks_level = 5
    with pytest.raises(tfhe_amd.TfheError) as ei:
        tfhe_amd.Engine(p, 0)
    assert ei.value.code == -5


def test_gl64_primitives_exact(tmp_path):
    """Goldilocks primitives of the device kernels (tfhe_amd/csrc/gl64.h, compiled for the host)
    against 128-bit reference arithmetic, including non-canonical inputs."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    exe = str(tmp_path / "gl64_check")
    subprocess.run([hipcc, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "tfhe_amd", "csrc"),
                    os.path.join(ROOT, "tools", "microbench", "gl64_check.cpp"), "-o", exe],
                   check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout


def test_ms_noise_reduction_rule_oracle(oracle_mod):
    """The oracle's modulus-switch noise reduction follows its stated rule (tfhe_oracle.h or_ms_key):
    brute-force every zero's measure and replay the sequential choice; the phase moves only by the
    zero's noise; the measure never grows."""
    prm = oracle_mod.params(1)
    ok = oracle_mod.Keys(prm, KEY_SEED, with_bsk=False)
    bound = oracle_mod.MS_FHEVM["bound"]
    msgs = (np.arange(24, dtype=np.uint64) % 16) * np.uint64((1 << 63) // 16)
    big = ok.encrypt(msgs, seed=0xC0FFEE31)
    small = np.stack([oracle_mod.keyswitch(prm, ok, c) for c in big])
    rng = np.random.default_rng(3)
    small[-2:] = rng.integers(0, 2 ** 64 - 1, size=(2, prm.n + 1), dtype=np.uint64)   # no zero reaches the bound
    red, picks = oracle_mod.ms_reduce(prm, ok, small)
    for q in range(small.shape[0]):
        best = oracle_mod.ms_measure(prm, ok, small[q])
        want = -1
        if best > bound:
            for z in range(ok.ms_zeros.shape[0]):
                m = oracle_mod.ms_measure(prm, ok, small[q], z)
                if m < best:
                    best, want = m, z
                    if best <= bound:
                        break
        assert picks[q] == want, q
        assert oracle_mod.ms_measure(prm, ok, red[q]) == best
        if want >= 0:
            assert np.array_equal(red[q], small[q] + ok.ms_zeros[want])
    assert (picks[:-2] >= 0).mean() > 0.5 and (picks[-2:] >= 0).all()
    d = (ok.phase(red[:-2], ok.lwe_key, prm.n) - ok.phase(small[:-2], ok.lwe_key, prm.n)).view(np.int64)
    assert np.abs(d).max() < 2 ** 50


def test_entropy_keygen_and_encryption_are_fresh():
    """no public default seed.  gen_keys / server_keygen / encrypt without a seed draw
    192 bits of OS entropy: two key sets, two server keys for one client key and two encryptions of
    one message all differ (and still decrypt); an explicit seed stays reproducible (tests, oracle)."""
    import tfhe_amd
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT)
    a, _ = tfhe_amd.gen_keys(p, with_server_key=False)
    b, _ = tfhe_amd.gen_keys(p, with_server_key=False)
    assert a.seed is None and not np.array_equal(a.lwe_key, b.lwe_key)
    s1, s2 = tfhe_amd.gen_keys(p, 99, with_server_key=False)[0], tfhe_amd.gen_keys(p, 99, with_server_key=False)[0]
    assert np.array_equal(s1.lwe_key, s2.lwe_key)
    c1, c2 = a.encrypt_bool([True, False]), a.encrypt_bool([True, False])
    assert not np.array_equal(c1, c2)
    assert list(a.decrypt_bool(c1)) == [True, False] and list(a.decrypt_bool(c2)) == [True, False]
    assert np.array_equal(a.encrypt_bool([True], seed=5), a.encrypt_bool([True], seed=5))
    k1, k2 = tfhe_amd.rng_key(), tfhe_amd.rng_key()
    assert list(k1.w) != list(k2.w)
    fh = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM)
    ck, _ = tfhe_amd.gen_keys(fh, 7, with_server_key=False)
    sk1, sk2 = tfhe_amd.server_keygen(ck), tfhe_amd.server_keygen(ck)
    assert not np.array_equal(sk1.ksk[:4096], sk2.ksk[:4096])
    assert not np.array_equal(sk1.ms_zeros[:4], sk2.ms_zeros[:4])
    # the KSK rows still encrypt the right key bits: phase of row (j=0, level 0) is s'_0 * 2^60 + small noise
    ph = ck.phase(sk1.ksk[: fh.n + 1], key=ck.lwe_key)
    want = int(ck.glwe_key[0]) << 60
    assert abs(((int(ph[0]) - want + (1 << 63)) % (1 << 64)) - (1 << 63)) < (1 << 50)
