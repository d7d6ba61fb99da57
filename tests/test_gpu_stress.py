"""Rare-failure screen: large batches through every blind-rotate kernel with every output decrypted.
A synchronization bug that corrupts ~1e-4 of PBS (as the LDS-DMA barrier race did, DESIGN.md §7b')
shows up here as several wrong decryptions; noise failures at these parameters are < 2^-60."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_stress_pgate_64k(engine, product_keys):
    ck, _ = product_keys
    B = 16384
    rng = np.random.default_rng(64)
    bits = rng.integers(0, 2, B).astype(bool)
    cts = ck.encrypt_bool(bits, seed=0x57E55)
    lut = engine.gate_lut()
    bad = 0
    for rep, thr in enumerate((0, 0, 1 << 30, 0)):   # batch kernel x3 (B > 4096), latency kernel x1
        engine.set_latency_batch(thr if thr else 0)
        out = engine.pbs(cts if rep % 2 == 0 else cts[::-1].copy(), lut)
        want = bits if rep % 2 == 0 else bits[::-1]
        bad += int(np.count_nonzero(ck.decrypt_bool(out) != want))
    engine.set_latency_batch(1024)
    assert bad == 0, f"{bad} wrong of {4 * B}"


def test_stress_pfhevm_16k(fhevm_engine, fhevm_keys):
    ck, _ = fhevm_keys
    B = 16384
    mm = 16
    rng = np.random.default_rng(16)
    msgs = rng.integers(0, mm, B).astype(np.uint64)
    cts = ck.encrypt(msgs, mm, seed=0x57E56)
    tabs = [[(m * (s + 3) + s) % mm for m in range(mm)] for s in range(5)]
    luts = np.stack([fhevm_engine.generate_accumulator(lambda m, t=t: t[m], mm) for t in tabs])
    idx = (np.arange(B) % 5).astype(np.uint32)
    out = fhevm_engine.pbs(cts, luts, idx)
    want = np.array([tabs[i][int(m)] for i, m in zip(idx, msgs)], dtype=np.uint64)
    assert np.count_nonzero(ck.decrypt(out, mm) != want) == 0


def test_stress_pgate_fft64_64k(gate_fft_engine, gate_fft_keys):
    """The headline kernel (FFT64 batch, blind_rotate_fft_pair_kernel): 4 x 16,384 PBS, every output decrypted;
    the last pass through the latency kernel."""
    ck, _ = gate_fft_keys
    B = 16384
    bits = np.random.default_rng(65).integers(0, 2, B).astype(bool)
    cts = ck.encrypt_bool(bits, seed=0x57E57)
    lut = gate_fft_engine.gate_lut()
    bad = 0
    try:
        for rep, thr in enumerate((0, 0, 0, 1 << 30)):
            gate_fft_engine.set_latency_batch(thr)
            out = gate_fft_engine.pbs(cts if rep % 2 == 0 else cts[::-1].copy(), lut)
            want = bits if rep % 2 == 0 else bits[::-1]
            bad += int(np.count_nonzero(ck.decrypt_bool(out) != want))
    finally:
        gate_fft_engine.set_latency_batch(256)
    assert bad == 0, f"{bad} wrong of {4 * B}"


def test_stress_pfhevm_fft64_64k(fhevm_fft_engine, fhevm_fft_keys):
    """P-FHEVM FFT64 kernels (blind_rotate_fft2k_kernel and the N = 2048 latency kernel): 4 x 16,384 PBS
    with five LUTs, every output decrypted."""
    ck, _ = fhevm_fft_keys
    B, mm = 16384, 16
    msgs = np.random.default_rng(17).integers(0, mm, B).astype(np.uint64)
    cts = ck.encrypt(msgs, mm, seed=0x57E58)
    tabs = [[(m * (s + 5) + 2 * s) % mm for m in range(mm)] for s in range(5)]
    luts = np.stack([fhevm_fft_engine.generate_accumulator(lambda m, t=t: t[m], mm) for t in tabs])
    bad = 0
    try:
        for rep, thr in enumerate((0, 0, 0, 1 << 30)):
            fhevm_fft_engine.set_latency_batch(thr)
            idx = ((np.arange(B) + rep) % 5).astype(np.uint32)
            out = fhevm_fft_engine.pbs(cts, luts, idx)
            want = np.array([tabs[i][int(m)] for i, m in zip(idx, msgs)], dtype=np.uint64)
            bad += int(np.count_nonzero(ck.decrypt(out, mm) != want))
    finally:
        fhevm_fft_engine.set_latency_batch(512)
    assert bad == 0, f"{bad} wrong of {4 * B}"
