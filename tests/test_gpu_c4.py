"""C4 at its size on one MI355X (BASELINE.json configs[3], SURVEY §8e: "batch=65536 PBS sharded across 8 GPUs,
BSK/KSK broadcast once"): one P-GATE FFT64 engine over EIGHT C-ABI shards of device 0
(tfhe_hip_create(params, {0 x 8}, 8)), keys uploaded once to shard 0 and replicated to the other seven by the
key-load broadcast (device copies: RCCL needs distinct ordinals; the N-rank RCCL call structure is
tests/test_bcast_plan.py), one global batch of 65,536 PBS split into eight contiguous 8,192-PBS slices run
concurrently.  Every output is decrypted; both sides of all seven shard boundaries are bit-exact against the
CPU oracle; a 4,096-PBS window straddling a boundary equals a single-shard engine's run of the same window."""
import time

import numpy as np
import pytest

import tfhe_amd

pytestmark = pytest.mark.gpu

G, SHARDS = 65536, 8
KEY_SEED = 0x7F4E0001


def test_c4_65536_over_eight_shards_one_gpu():
    from oracle import oracle as O
    params = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT)
    ck, sk = tfhe_amd.gen_keys(params, KEY_SEED)
    bits = np.random.default_rng(0xC4).integers(0, 2, G).astype(bool)
    cts = ck.encrypt_bool(bits, seed=0xC0FFEE04)
    with tfhe_amd.Engine(params, [0] * SHARDS) as eng:
        eng.load_keys(sk)
        assert eng.key_bcast_mode == "copy"
        assert tfhe_amd.lib().tfhe_hip_ndev(eng._h) == SHARDS
        lut = eng.gate_lut()
        eng.pbs(cts[:SHARDS * 64], lut)                        # warm every shard
        t = time.time()
        out = eng.pbs(cts, lut)
        dt = time.time() - t
    print(f"C4 on one GPU: {G} PBS over {SHARDS} shards in {dt * 1e3:.1f} ms (host buffers incl. H2D/D2H): "
          f"{G / dt:.0f} PBS/s")
    assert np.array_equal(ck.decrypt_bool(out), bits)          # every one of the 65,536 outputs
    bounds = [G * s // SHARDS for s in range(1, SHARDS)]
    sel = np.array([0] + [b + d for b in bounds for d in (-1, 0)] + [G - 1])
    prm = O.params(tfhe_amd.PRESET_GATE_FFT)
    keys = O.Keys(prm, KEY_SEED)
    ref = O.pbs_batch_fft(prm, keys, cts[sel], O.lut_constant(1024, O.MU)[None], threads=8)
    assert np.array_equal(out[sel], ref)
    lo = bounds[2] - 2048                                      # window [22528, 26624) straddles shards 2 | 3
    with tfhe_amd.Engine(params, 0) as one:
        one.load_keys(sk)
        assert np.array_equal(one.pbs(cts[lo:lo + 4096], one.gate_lut()), out[lo:lo + 4096])
