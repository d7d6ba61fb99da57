"""The key-load broadcast planner (tfhe_hip_bcast_plan, api.cpp:bcast_plan) on CPU: the N-rank call
structure tfhe_hip_load_keys issues over a multi-device engine, checked without N GPUs (one
ncclBroadcast of BSK / KSK from device 0; the one-GPU box only ever runs N = 1 or repeated ordinals)."""
import ctypes

import pytest

import tfhe_amd

MODE_NONE, MODE_COPY, MODE_RCCL = 0, 1, 2


def plan(devices, policy=None, rccl=True):
    L = tfhe_amd.lib()
    L.tfhe_hip_bcast_plan.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    devs = (ctypes.c_int * len(devices))(*devices)
    calls = (ctypes.c_int * 16)()
    mode = ctypes.c_int(-1)
    n = L.tfhe_hip_bcast_plan(devs, len(devices), None if policy is None else policy.encode(), int(rccl),
                              ctypes.byref(mode), calls, 16)
    return n, mode.value, list(calls[:max(n, 0)])


@pytest.mark.parametrize("nd", [2, 4, 8])
def test_rccl_group_covers_every_rank_root_first(nd):
    n, mode, calls = plan(list(range(nd)))
    assert mode == MODE_RCCL and n == nd
    assert calls == list(range(nd))          # one ncclBroadcast per rank in one group, root 0 first


def test_single_device_needs_nothing_unless_forced():
    assert plan([0])[:2] == (0, MODE_NONE)
    assert plan([0], "rccl") == (1, MODE_RCCL, [0])   # the one-device RCCL plumbing test (test_gpu_multidev)


def test_repeated_ordinals_use_device_copies():
    n, mode, calls = plan([0] * 8)
    assert mode == MODE_COPY and calls == list(range(1, 8))   # C4 on one GPU: 7 copies from shard 0
    assert plan([0, 0], "rccl")[0] < 0                       # RCCL cannot span a repeated ordinal


def test_missing_rccl_falls_back_to_peer_copies():
    n, mode, calls = plan([0, 1, 2, 3], rccl=False)
    assert mode == MODE_COPY and calls == [1, 2, 3]
    assert plan([0, 1], "rccl", rccl=False)[0] < 0           # forced RCCL without the library is an error
    assert plan([0, 1], "copy")[1] == MODE_COPY
    assert plan([0, 1], "bogus")[0] < 0
