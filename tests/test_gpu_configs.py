"""BASELINE.json configs C3 and C5 as MI355X parity cases.

C3: "FheUint8 LUT eval (8 PBS per ciphertext), batch=4096" — 4096 FheUint8 values, each bit
    bootstrapped with its own LUT (lut_index = bit position): 32,768 PBS in one launch; every
    decrypted byte checked, a sample bit-exact against the oracle.
C5: "FheUint32 comparison tree, 256 bidders" — tfhe_amd.auction.max_tree: 255 FheUint32 max
    comparisons in 8 dependent levels (lockstep per level), with the winner's index.
"""
import time

import numpy as np
import pytest

import tfhe_amd
from tfhe_amd import integer as I
from tfhe_amd.auction import max_tree

pytestmark = pytest.mark.gpu
P = 0xFFFFFFFF00000001


@pytest.mark.parametrize("transform", ["ntt", "fft64"])
def test_c3_fheuint8_lut_eval_4096(request, transform, oracle_mod):
    """C3 on both engines: the FFT64 engine is the default of the bench and of the JS binding."""
    engine = request.getfixturevalue("engine" if transform == "ntt" else "gate_fft_engine")
    ck, _ = request.getfixturevalue("product_keys" if transform == "ntt" else "gate_fft_keys")
    if transform == "ntt":
        gate_params, oracle_keys = request.getfixturevalue("gate_params"), request.getfixturevalue("oracle_keys")
    else:
        gate_params = oracle_mod.params(tfhe_amd.PRESET_GATE_FFT)
        oracle_keys = oracle_mod.Keys(gate_params, 0x7F4E0001)
    B = 4096
    rng = np.random.default_rng(3)
    vals = rng.integers(0, 256, B).astype(np.uint64)
    X = tfhe_amd.FheUint8.encrypt(vals, ck, engine, seed=0xC0FFEE03)
    gate = engine.gate_lut()
    inv = (np.uint64(0) - gate.astype(np.uint64)) % np.uint64(P)      # LUT == -1/8: NOT
    mask = 0b10110010
    luts = np.stack([inv if (mask >> j) & 1 else gate for j in range(8)])   # 8 per-bit LUTs
    Y = X.map_bits(luts)
    assert np.array_equal(Y.decrypt(ck), vals ^ np.uint64(mask))
    # sampled bit-exact parity: bits of 4 values through the oracle with the same LUT table / index
    sel = np.array([0, 1, 2047, 4095])
    cts = X.bits[sel].reshape(-1, X.bits.shape[-1])
    idx = np.tile(np.arange(8, dtype=np.uint32), len(sel))
    ref = oracle_mod.pbs_batch(gate_params, oracle_keys, cts, luts, idx)
    assert np.array_equal(Y.bits[sel].reshape(-1, X.bits.shape[-1]), ref)


@pytest.mark.parametrize("transform", ["ntt", "fft64"])
def test_c5_auction_max_tree_256(request, transform):
    engine = request.getfixturevalue("engine" if transform == "ntt" else "gate_fft_engine")
    ck, _ = request.getfixturevalue("product_keys" if transform == "ntt" else "gate_fft_keys")
    B = 256
    t0 = time.time()
    v = np.random.default_rng(5).integers(0, 2**32, B, dtype=np.uint64)
    v[77] = v[200] = np.uint64(2**32 - 3)            # tie at the top: the lower index wins
    c = I.Circuit(engine)
    bids = I.FheUint.encrypt(c, ck, v, 32, seed=0xB1D, stream0=0)
    mx, idx = max_tree(c, bids)
    assert int(mx.decrypt(ck)[0]) == 2**32 - 3
    assert int(idx.decrypt(ck)[0]) == 77
    assert c.pbs_count > 255 * 100                   # really ran the comparator circuits
    print(f"C5 {transform}: {time.time() - t0:.2f} s, {c.pbs_count} PBS in {c.launches} launches")


def test_c5_device_resident_equals_host(gate_fft_engine, gate_fft_keys):
    """C5 on the device-resident circuit (Circuit(device=...): int64 tensors on the GPU, every level one
    pbs_async on torch's stream): the same winner, the same launches and PBS count, and every output bit of the
    max equal to the host-array circuit's (same keys, same encryptions, deterministic kernels)."""
    import torch
    ck, _ = gate_fft_keys
    v = np.random.default_rng(6).integers(0, 2**32, 256, dtype=np.uint64)
    out = []
    for dev in (None, "cuda:0"):
        c = I.Circuit(gate_fft_engine, device=dev)
        bids = I.FheUint.encrypt(c, ck, v, 32, seed=0xB1E, stream0=0)
        t0 = time.time()
        mx, idx = max_tree(c, bids)
        if dev:
            torch.cuda.synchronize()
        wall = time.time() - t0
        bits = mx.bits.cpu().numpy().view(np.uint64) if dev else mx.bits
        out.append((bits, c.launches, c.pbs_count, int(mx.decrypt(ck)[0]), int(idx.decrypt(ck)[0])))
        print(f"C5 fft64 {'device' if dev else 'host'}: {wall:.3f} s")
    assert out[0][3:] == out[1][3:] == (int(v.max()), int(np.argmax(v)))
    assert out[0][1:3] == out[1][1:3]
    assert np.array_equal(out[0][0], out[1][0])


@pytest.mark.parametrize("transform", ["ntt", "fft64"])
def test_c2_batch_1024(request, transform, oracle_mod):
    """C2: batch = 1024 independent P-GATE PBS on one GPU (the exact config size: the FFT64 engine runs
    its batch kernel here, the NTT engine its latency kernel), every output decrypted, a sample of 16
    bit-exact against the oracle."""
    engine = request.getfixturevalue("engine" if transform == "ntt" else "gate_fft_engine")
    ck, _ = request.getfixturevalue("product_keys" if transform == "ntt" else "gate_fft_keys")
    B = 1024
    bits = np.random.default_rng(0xC2).integers(0, 2, B).astype(bool)
    cts = ck.encrypt_bool(bits, seed=0xC0FFEE02)
    lut = engine.gate_lut()
    out = engine.pbs(cts, lut)
    assert np.array_equal(ck.decrypt_bool(out), bits)
    preset = tfhe_amd.PRESET_GATE if transform == "ntt" else tfhe_amd.PRESET_GATE_FFT
    prm = oracle_mod.params(preset)
    keys = request.getfixturevalue("oracle_keys") if transform == "ntt" else oracle_mod.Keys(prm, 0x7F4E0001)
    sel = np.linspace(0, B - 1, 16).astype(int)
    assert np.array_equal(out[sel], oracle_mod.pbs_batch(prm, keys, cts[sel], lut[None]))
