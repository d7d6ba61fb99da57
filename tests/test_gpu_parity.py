"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit-exact.

Sizes are small enough for the oracle to finish in seconds; the batch-4096 test checks
size-independent properties (every output decrypts correctly) plus a sampled bit-exact subset.
"""
import hashlib

import numpy as np
import pytest

from conftest import load_golden

import tfhe_amd

pytestmark = pytest.mark.gpu
P = 0xFFFFFFFF00000001


def test_ntt_forward_inverse_vs_oracle(engine, oracle_mod):
    g = load_golden("ntt_1024.npz")
    assert np.array_equal(engine.ntt_fwd(g["input"]), g["output"])
    rng = np.random.default_rng(11)
    x = rng.integers(0, P, size=(33, 1024), dtype=np.uint64)
    X = engine.ntt_fwd(x)
    assert np.array_equal(X, oracle_mod.ntt_fwd(x))
    assert np.array_equal(engine.ntt_inv(X), x)
    assert np.array_equal(engine.ntt_inv(x), oracle_mod.ntt_inv(x))


def test_golden_pbs_stages(engine):
    g = load_golden("pbs_gate.npz")
    acc = engine.blind_rotate(g["lwe_in"][:1], g["luts"][:1])
    assert np.array_equal(acc[0], g["acc0"]), "blind rotation differs from the oracle"
    assert np.array_equal(engine.sample_extract(g["acc0"][None])[0], g["big0"])
    assert np.array_equal(engine.keyswitch(g["big0"][None])[0], g["ks0"])
    out = engine.pbs(g["lwe_in"], g["luts"], g["lut_index"])
    assert np.array_equal(out, g["lwe_out"])


def test_golden_nand(engine, product_keys):
    ck, _ = product_keys
    g = load_golden("nand_gate.npz")
    out = engine.nand(g["c1"], g["c2"])
    assert np.array_equal(out, g["out"])
    assert np.array_equal(ck.decrypt_bool(out).astype(np.uint8), g["expect"])


def test_golden_batch_digest(engine, product_keys):
    ck, _ = product_keys
    g = load_golden("pbs_batch64.npz")
    cts = ck.encrypt_torus(g["msgs"], seed=int(g["input_seed"]))
    assert hashlib.sha256(cts.tobytes()).digest() == g["sha256_in"].tobytes()
    out = engine.pbs(cts, engine.gate_lut())
    assert hashlib.sha256(out.tobytes()).digest() == g["sha256_out"].tobytes()


def test_blind_rotate_vs_oracle_random(engine, product_keys, oracle_mod, gate_params, oracle_keys):
    ck, _ = product_keys
    rng = np.random.default_rng(5)
    cts = ck.encrypt_torus(rng.integers(0, 2**63, 3, dtype=np.uint64), seed=77)
    lut = oracle_mod.lut_from_table(1024, 8, list(range(8)), (1 << 63) // 8)
    acc = engine.blind_rotate(cts, lut)
    for i in range(3):
        assert np.array_equal(acc[i], oracle_mod.blind_rotate(gate_params, oracle_keys, cts[i], lut))


def test_keyswitch_vs_oracle(engine, oracle_mod, gate_params, oracle_keys):
    rng = np.random.default_rng(9)
    big = rng.integers(0, 2**64 - 1, size=(70, 1025), dtype=np.uint64)  # crosses a 64-ciphertext tile
    out = engine.keyswitch(big)
    for i in (0, 1, 63, 64, 69):
        assert np.array_equal(out[i], oracle_mod.keyswitch(gate_params, oracle_keys, big[i]))


def test_pbs_vs_oracle_multi_lut(engine, product_keys, oracle_mod, gate_params, oracle_keys):
    ck, _ = product_keys
    B = 24
    rng = np.random.default_rng(21)
    msgs = rng.integers(0, 4, B).astype(np.uint64) * np.uint64(1 << 61)
    cts = ck.encrypt_torus(msgs, seed=0xC0FFEE10)
    luts = np.stack([oracle_mod.lut_from_table(1024, 4, [(m + s) % 4 for m in range(4)], 1 << 61) for s in range(4)])
    idx = rng.integers(0, 4, B).astype(np.uint32)
    out = engine.pbs(cts, luts, idx)
    ref = oracle_mod.pbs_batch(gate_params, oracle_keys, cts, luts, idx)
    assert np.array_equal(out, ref)
    dec = ck.decrypt(out, 4)
    assert np.array_equal(dec, (msgs // np.uint64(1 << 61) + idx) % 4)


@pytest.mark.parametrize("msg_modulus", [4, 8])
def test_lut_all_messages_popcount(engine, product_keys, msg_modulus):
    """biometrics main.rs:65-77: decrypt(keyswitch_programmable_bootstrap(ct, acc(f))) == f(m)."""
    ck, _ = product_keys
    f = lambda m: bin(m).count("1")
    msgs = np.arange(msg_modulus)
    cts = ck.encrypt(np.repeat(msgs, 4), msg_modulus, seed=3)
    acc = engine.generate_accumulator(f, msg_modulus)
    out = engine.keyswitch_programmable_bootstrap(cts, acc)
    assert np.array_equal(ck.decrypt(out, msg_modulus), np.repeat([f(m) % msg_modulus for m in msgs], 4))


def test_fhebool_gates(engine, product_keys):
    ck, _ = product_keys
    a = np.array([0, 0, 1, 1] * 4, dtype=bool)
    b = np.array([0, 1, 0, 1] * 4, dtype=bool)
    A = tfhe_amd.FheBool.encrypt(a, ck, engine, seed=1)
    Bb = tfhe_amd.FheBool.encrypt(b, ck, engine, seed=2)
    assert np.array_equal(A.nand(Bb).decrypt(ck), ~(a & b))
    assert np.array_equal((A & Bb).decrypt(ck), a & b)
    assert np.array_equal((A | Bb).decrypt(ck), a | b)
    assert np.array_equal((A ^ Bb).decrypt(ck), a ^ b)
    assert np.array_equal((~A).decrypt(ck), ~a)
    # depth: 20 chained NANDs stay correct (noise is refreshed by every bootstrap)
    x, y = A, Bb
    ref_x, ref_y = a, b
    for _ in range(20):
        x, y = x.nand(y), x
        ref_x, ref_y = ~(ref_x & ref_y), ref_x
    assert np.array_equal(x.decrypt(ck), ref_x)


def test_fheuint8_map_bits(engine, product_keys):
    ck, _ = product_keys
    vals = np.array([0, 1, 71, 66, 137, 255, 128, 200], dtype=np.uint64)
    X = tfhe_amd.FheUint8.encrypt(vals, ck, engine, seed=4)
    gate = engine.gate_lut()
    inv = (np.uint64(0) - gate.astype(np.uint64)) % np.uint64(P)  # LUT == -1/8: negates the bit
    luts = np.stack([inv if j % 2 == 0 else gate for j in range(8)])
    assert np.array_equal(X.map_bits(luts).decrypt(ck), vals ^ np.uint64(0x55))
    assert np.array_equal(X.refresh().decrypt(ck), vals)


def test_batch_4096_properties_and_sampled_parity(engine, product_keys, oracle_mod, gate_params, oracle_keys):
    ck, _ = product_keys
    B = 4096
    rng = np.random.default_rng(4096)
    bits = rng.integers(0, 2, B).astype(bool)
    cts = ck.encrypt_bool(bits, seed=0xC0FFEE02)
    out = engine.pbs(cts, engine.gate_lut())
    assert np.array_equal(ck.decrypt_bool(out), bits)
    sample = rng.choice(B, 32, replace=False)
    ref = oracle_mod.pbs_batch(gate_params, oracle_keys, cts[sample], oracle_mod.lut_constant(1024, oracle_mod.MU)[None])
    assert np.array_equal(out[sample], ref)


def test_edge_cases(engine, product_keys, oracle_mod, gate_params, oracle_keys):
    ck, _ = product_keys
    gate = engine.gate_lut()
    # empty batch is a no-op
    assert engine.pbs(np.zeros((0, 631), dtype=np.uint64), gate).shape == (0, 631)
    # trivial ciphertexts: zero mask (every mod-switched a_i == 0 -> the CMUX loop is skipped)
    triv = np.zeros((3, 631), dtype=np.uint64)
    triv[:, 630] = [1 << 61, (1 << 64) - (1 << 61), (1 << 63) - 1]
    out = engine.pbs(triv, gate)
    ref = oracle_mod.pbs_batch(gate_params, oracle_keys, triv, gate[None])
    assert np.array_equal(out, ref)
    # mask values on the rounding boundaries of the modulus switch
    edge = np.zeros((2, 631), dtype=np.uint64)
    edge[0, :630] = np.uint64((1 << 52) - 1)
    edge[1, :630] = np.uint64((1 << 64) - (1 << 52))
    edge[:, 630] = 1 << 61
    assert np.array_equal(engine.pbs(edge, gate), oracle_mod.pbs_batch(gate_params, oracle_keys, edge, gate[None]))
    # bad lut_index -> EINVAL, nothing launched
    with pytest.raises(tfhe_amd.TfheError) as e:
        engine.pbs(triv, gate, lut_index=[0, 1, 0])
    assert e.value.code == -1


def test_no_keys_is_an_error():
    eng = tfhe_amd.Engine(tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE), 0)
    with pytest.raises(tfhe_amd.TfheError) as e:
        eng.pbs(np.zeros((1, 631), dtype=np.uint64), tfhe_amd.lut_constant(1024, 1 << 61))
    assert e.value.code == -4
    eng.close()


def test_device_resident_async_and_device_keys(engine, product_keys):
    """pbs_async on torch tensors (inputs resident in HBM) and keys loaded from device buffers
    (the path used after an RCCL broadcast) give the same bytes as the host path."""
    import torch
    ck, sk = product_keys
    cts = ck.encrypt_bool(np.arange(100) % 3 == 0, seed=12)
    ref = engine.pbs(cts, engine.gate_lut())
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(cts.view(np.int64)).to(dev)
    d_lut = torch.from_numpy(engine.gate_lut().view(np.int64)).to(dev)
    d_out = torch.empty_like(d_in)
    eng2 = tfhe_amd.Engine(ck.params, 0)
    eng2.load_keys_device(torch.from_numpy(sk.bsk.view(np.int64)).to(dev), torch.from_numpy(sk.ksk.view(np.int64)).to(dev))
    eng2.pbs_async(d_in, d_lut, d_out)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy().view(np.uint64), ref)
    # ordered with torch's default stream without an explicit device synchronize
    d_out2 = torch.zeros_like(d_in)
    eng2.pbs_async(d_in, d_lut, d_out2)
    assert np.array_equal(d_out2.cpu().numpy().view(np.uint64), ref)
    eng2.close()


@pytest.mark.parametrize("B", [1, 37, 300])
def test_latency_and_batch_kernels_agree(engine, product_keys, oracle_mod, gate_params, oracle_keys, B):
    """The latency kernel (one ciphertext per workgroup) and the batch kernel (8 per workgroup) are
    bit-identical, and both equal the oracle on a sample."""
    ck, _ = product_keys
    rng = np.random.default_rng(B)
    msgs = rng.integers(0, 8, B).astype(np.uint64) * np.uint64(1 << 60)
    cts = ck.encrypt_torus(msgs, seed=0xC0FFEE30 + B)
    lut = oracle_mod.lut_from_table(1024, 8, [(5 * m + 3) % 8 for m in range(8)], 1 << 60)
    try:
        engine.set_latency_batch(0)
        acc_b = engine.blind_rotate(cts, lut)
        out_b = engine.pbs(cts, lut)
        engine.set_latency_batch(1 << 20)
        acc_l = engine.blind_rotate(cts, lut)
        out_l = engine.pbs(cts, lut)
    finally:
        engine.set_latency_batch(1024)
    assert np.array_equal(acc_l, acc_b)
    assert np.array_equal(out_l, out_b)
    i = B // 2
    assert np.array_equal(acc_l[i], oracle_mod.blind_rotate(gate_params, oracle_keys, cts[i], lut))
