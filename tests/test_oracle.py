"""CPU oracle self-checks and golden-vector pinning (no GPU).

The oracle (oracle/tfhe_oracle.c) is the bit-exact checker for the HIP path.  Ciphertext-level
parity with the reference's absent tfhe-rs core is "parity unpinned"; what IS pinned here:
  * the NTT against the O(N^2) schoolbook product and the definition A[j] = a(psi^(2j+1));
  * the decomposition against its recomposition bound (tfhe-rs SignedDecomposer semantics);
  * message-level KATs: NAND truth table, decrypt(PBS(f)) == f(m) for every message
    (ml/biometrics/notebooks/main.rs:65-77 pattern);
  * the committed golden fixtures (tests/golden/make_golden.py).
"""
import hashlib

import numpy as np
import pytest

from conftest import KEY_SEED, load_golden

P = 0xFFFFFFFF00000001


@pytest.mark.parametrize("N", [32, 64, 1024, 2048])
def test_ntt_matches_schoolbook(oracle_mod, N):
    O = oracle_mod
    rng = np.random.default_rng(N)
    a = rng.integers(0, P, N, dtype=np.uint64)
    b = rng.integers(0, P, N, dtype=np.uint64)
    assert np.array_equal(O.poly_mul_schoolbook(a, b), O.poly_mul_ntt(a, b))
    assert np.array_equal(O.ntt_inv(O.ntt_fwd(a)), a)


def test_ntt_definition(oracle_mod):
    O = oracle_mod
    N = 1024
    psi = O.psi(N)
    assert pow(psi, 32, P) == 8 and pow(psi, N, P) == P - 1
    a = np.random.default_rng(7).integers(0, P, N, dtype=np.uint64)
    A = O.ntt_fwd(a)
    for j in (0, 3, 511, 1023):
        assert int(A[j]) == sum(int(a[i]) * pow(psi, (2 * j + 1) * i, P) for i in range(N)) % P


def test_golden_ntt(oracle_mod):
    g = load_golden("ntt_1024.npz")
    assert np.array_equal(oracle_mod.ntt_fwd(g["input"]), g["output"])
    assert int(g["psi"]) == oracle_mod.psi(1024)
    assert np.all(g["output"][0] == 1)  # NTT of the constant 1


@pytest.mark.parametrize("base_log,level", [(7, 3), (2, 8), (23, 1), (4, 4)])
def test_decomposition_recomposes(oracle_mod, base_log, level):
    O = oracle_mod
    rng = np.random.default_rng(base_log * 100 + level)
    B = 1 << base_log
    prec = base_log * level
    for x in list(rng.integers(0, 2**63, 200, dtype=np.uint64)) + [0, 2**64 - 1, 2**63, 2**(64 - prec - 1)]:
        x = int(x)
        d = O.decompose(x, base_log, level)
        assert all(-B // 2 <= v <= B // 2 for v in d)
        rec = sum(v << (64 - base_log * (l + 1)) for l, v in enumerate(d)) % (1 << 64)
        err = (rec - x) % (1 << 64)
        err = min(err, (1 << 64) - err)
        assert err <= 1 << (64 - prec - 1)


def test_mod_switch(oracle_mod):
    L = oracle_mod.lib()
    assert L.or_mod_switch(0, 2048) == 0
    assert L.or_mod_switch(1 << 63, 2048) == 1024
    assert L.or_mod_switch((1 << 52), 2048) == 1  # exactly half a step rounds up
    assert L.or_mod_switch((1 << 64) - 1, 2048) == 0


def test_nand_truth_table(oracle_mod, gate_params, oracle_keys):
    O = oracle_mod
    g = load_golden("nand_gate.npz")
    for i in range(4):
        out = O.nand(gate_params, oracle_keys, g["c1"][i], g["c2"][i])
        assert np.array_equal(out, g["out"][i]), "oracle drifted from the golden NAND vector"
        assert O.decode_bit(int(oracle_keys.phase(out)[0])) == int(g["expect"][i])


def test_golden_pbs(oracle_mod, gate_params, oracle_keys):
    O = oracle_mod
    g = load_golden("pbs_gate.npz")
    assert int(g["key_seed"]) == KEY_SEED
    out = O.pbs_batch(gate_params, oracle_keys, g["lwe_in"], g["luts"], g["lut_index"])
    assert np.array_equal(out, g["lwe_out"])
    acc = O.blind_rotate(gate_params, oracle_keys, g["lwe_in"][0], g["luts"][0])
    assert np.array_equal(acc, g["acc0"])
    assert np.array_equal(O.sample_extract(gate_params, acc), g["big0"])
    assert np.array_equal(O.keyswitch(gate_params, oracle_keys, g["big0"]), g["ks0"])


def test_golden_batch_digest(oracle_mod, gate_params, oracle_keys):
    O = oracle_mod
    g = load_golden("pbs_batch64.npz")
    cts = oracle_keys.encrypt(g["msgs"], seed=int(g["input_seed"]))
    assert hashlib.sha256(cts.tobytes()).digest() == g["sha256_in"].tobytes()
    out = O.pbs_batch(gate_params, oracle_keys, cts, O.lut_constant(1024, O.MU)[None])
    assert hashlib.sha256(out.tobytes()).digest() == g["sha256_out"].tobytes()
    # every output decrypts to the input bit (identity gate LUT)
    assert np.array_equal(O.decode_bit(0) * 0 + (oracle_keys.phase(out) < (1 << 63)),
                          g["msgs"] == np.uint64(O.MU))


@pytest.mark.parametrize("msg_modulus,f", [(4, lambda m: (m * m + 1) % 4), (8, lambda m: bin(m).count("1"))])
def test_lut_pbs_all_messages(oracle_mod, gate_params, oracle_keys, msg_modulus, f):
    """decrypt(PBS(encrypt(m), LUT f)) == f(m) for every m (biometrics main.rs:65-77 KAT)."""
    O = oracle_mod
    delta = (1 << 63) // msg_modulus
    msgs = np.arange(msg_modulus, dtype=np.uint64) * np.uint64(delta)
    cts = oracle_keys.encrypt(msgs, seed=99, stream0=msg_modulus)
    lut = O.lut_from_table(1024, msg_modulus, [f(m) for m in range(msg_modulus)], delta)
    out = O.pbs_batch(gate_params, oracle_keys, cts, lut[None])
    ph = oracle_keys.phase(out).astype(object)
    dec = [((int(v) + delta // 2) // delta) % msg_modulus for v in ph]
    assert dec == [f(m) for m in range(msg_modulus)]


def test_blind_rotate_ntt_equals_schoolbook_small(oracle_mod):
    """The NTT blind rotation equals the schoolbook one (tiny parameter set: n=4, N=64)."""
    O = oracle_mod
    prm = O.Params(n=4, k=1, N=64, pbs_base_log=7, pbs_level=3, ks_base_log=2, ks_level=8,
                   lwe_noise_log2=-15, glwe_noise_log2=-25, order=0)
    keys = O.Keys(prm, 5)
    ct = keys.encrypt([1 << 61], seed=3)[0]
    lut = O.lut_constant(64, 1 << 61)
    a = O.blind_rotate(prm, keys, ct, lut, schoolbook=False)
    b = O.blind_rotate(prm, keys, ct, lut, schoolbook=True)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("name", ["fft64_gate.npz", "fft64_fhevm.npz"])
def test_golden_fft64(oracle_mod, name):
    """The FFT64 oracle (fft_oracle.c, the device's bit-exact twin) against its committed fixtures
    (tests/golden/make_golden_fft64.py): a lockstep edit of kernel and oracle changes these bytes."""
    g = load_golden(name)
    prm = oracle_mod.params(int(g["preset"]))
    keys = oracle_mod.Keys(prm, int(g["key_seed"]))
    bri = g["small"] if "small" in g else g["lwe_in"]
    if "small" in g:
        for i in range(bri.shape[0]):
            assert np.array_equal(oracle_mod.keyswitch(prm, keys, g["lwe_in"][i]), bri[i])
    for i in range(bri.shape[0]):
        acc = oracle_mod.blind_rotate_fft(prm, keys, bri[i], g["luts"][g["lut_index"][i]])
        assert np.array_equal(acc, g["acc"][i]), f"{name}: accumulator {i} drifted"
    out = oracle_mod.pbs_batch_fft(prm, keys, g["lwe_in"], g["luts"], g["lut_index"])
    assert np.array_equal(out, g["lwe_out"]), f"{name}: PBS output drifted"
