"""The multi-device C ABI (include/tfhe_hip.h: tfhe_hip_create(params, devices, ndev)) on a one-GPU box:
two shards of device 0 split every host batch and get their keys by device copy; a forced one-rank RCCL
communicator exercises the in-library RCCL broadcast plumbing (librccl loaded on first use); and
tfhe_hip_pbs_async on a side stream interleaved with synchronous calls on the ctx stream keeps the
shared workspaces ordered.  Results must equal the single-shard engine bit for bit."""
import os

import numpy as np
import pytest

import tfhe_amd

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset", [tfhe_amd.PRESET_GATE_FFT, tfhe_amd.PRESET_FHEVM_FFT, tfhe_amd.PRESET_GATE])
def test_two_shards_split_bitexact(preset):
    params = tfhe_amd.Params.preset(preset)
    ck, sk = tfhe_amd.gen_keys(params, 0x7F4E0001)
    B = 777                                                   # ragged: 388 + 389
    if params.order == 1:
        msgs = np.random.default_rng(1).integers(0, 16, B).astype(np.uint64)
        cts = ck.encrypt(msgs, 16, seed=11)
    else:
        bits = np.random.default_rng(1).integers(0, 2, B).astype(bool)
        cts = ck.encrypt_bool(bits, seed=11)
    with tfhe_amd.Engine(params, 0) as one, tfhe_amd.Engine(params, [0, 0]) as two:
        one.load_keys(sk)
        two.load_keys(sk)
        assert one.key_bcast_mode == "single" and two.key_bcast_mode == "copy"
        assert tfhe_amd.lib().tfhe_hip_ndev(two._h) == 2
        lut = one.generate_accumulator(lambda m: (5 * m + 3) % 16, 16) if params.order == 1 else one.gate_lut()
        ref = one.pbs(cts, lut)
        out = two.pbs(cts, lut)
        assert np.array_equal(out, ref)
        if params.order == 1:
            assert np.array_equal(ck.decrypt(out, 16), (5 * msgs + 3) % 16)
        else:
            assert np.array_equal(ck.decrypt_bool(out), bits)
            assert np.array_equal(two.nand(cts[:100], cts[100:200]), one.nand(cts[:100], cts[100:200]))


def test_rccl_broadcast_plumbing(monkeypatch):
    """TFHE_HIP_BCAST=rccl: keys go through ncclCommInitAll + ncclBroadcast even with one device."""
    params = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT)
    ck, sk = tfhe_amd.gen_keys(params, 0x7F4E0001)
    bits = np.random.default_rng(2).integers(0, 2, 64).astype(bool)
    cts = ck.encrypt_bool(bits, seed=12)
    monkeypatch.setenv("TFHE_HIP_BCAST", "rccl")
    with tfhe_amd.Engine(params, [0]) as eng:
        eng.load_keys(sk)
        assert eng.key_bcast_mode == "rccl"
        assert np.array_equal(ck.decrypt_bool(eng.pbs(cts, eng.gate_lut())), bits)


def test_async_side_stream_then_sync_call_ordered():
    """pbs_async on a torch side stream, then (without waiting) synchronous pbs / keyswitch calls on the
    ctx stream: the second user of the workspaces waits for the first, so both results are right."""
    import torch
    params = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT)
    ck, sk = tfhe_amd.gen_keys(params, 0x7F4E0001)
    B = 2048
    rng = np.random.default_rng(3)
    b1, b2 = rng.integers(0, 2, B).astype(bool), rng.integers(0, 2, B).astype(bool)
    c1, c2 = ck.encrypt_bool(b1, seed=13), ck.encrypt_bool(b2, seed=14)
    with tfhe_amd.Engine(params, 0) as eng:
        eng.load_keys(sk)
        dev = torch.device("cuda", 0)
        d_in = torch.from_numpy(c1.view(np.int64)).to(dev)
        d_lut = torch.from_numpy(eng.gate_lut().view(np.int64)).to(dev)
        d_out = torch.empty_like(d_in)
        side = torch.cuda.Stream(dev)
        torch.cuda.synchronize()
        for _ in range(3):
            eng.pbs_async(d_in, d_lut, d_out, stream=side)  # in flight on the side stream
            out2 = eng.pbs(c2, eng.gate_lut())                # ctx stream, same workspaces
            side.synchronize()
            assert np.array_equal(ck.decrypt_bool(d_out.cpu().numpy().view(np.uint64)), b1)
            assert np.array_equal(ck.decrypt_bool(out2), b2)
