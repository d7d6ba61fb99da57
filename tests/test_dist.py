"""World-size-2 gloo tests (CPU) of the multi-GPU plumbing in tfhe_amd/dist.py: sharding, the
one-time key broadcast, and the shard -> all_gather used between levels of chained circuits.
The per-rank "kernel" here is a deterministic CPU stand-in: the HIP path itself is covered by the
gpu tests; this checks that the N>1 data movement is correct by construction."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tfhe_amd.dist import broadcast_keys, shard_range, sharded_map, tree_levels


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # 1. key broadcast: rank 0 holds the keys, others receive them bit-exactly
        rng = np.random.default_rng(1234)
        bsk_ref = rng.integers(-2**62, 2**62, 4096, dtype=np.int64)
        ksk_ref = rng.integers(-2**62, 2**62, 1024, dtype=np.int64)
        if rank == 0:
            bsk, ksk = torch.from_numpy(bsk_ref.copy()), torch.from_numpy(ksk_ref.copy())
        else:
            bsk, ksk = torch.zeros(4096, dtype=torch.int64), torch.zeros(1024, dtype=torch.int64)
        broadcast_keys(bsk, ksk, src=0)
        ok_keys = bool(np.array_equal(bsk.numpy(), bsk_ref) and np.array_equal(ksk.numpy(), ksk_ref))
        # 2. sharded map + gather over a ragged global batch (7 rows over 2 ranks)
        g = torch.arange(7 * 3, dtype=torch.int64).reshape(7, 3)
        out = sharded_map(g, lambda x: x * 2 + 1)
        ok_map = bool(torch.equal(out, g * 2 + 1))
        # 3. chained tree (max over 256 "bidders" in 8 levels) with a gather per level
        vals = torch.from_numpy(np.random.default_rng(7).integers(0, 2**31, 256, dtype=np.int64)).reshape(-1, 1)
        cur = vals
        for _ in tree_levels(256):
            pairs = cur.reshape(-1, 2)
            cur = sharded_map(pairs, lambda p: p.max(dim=1, keepdim=True).values)
        ok_tree = int(cur.item()) == int(vals.max().item())
        q.put((rank, ok_keys, ok_map, ok_tree))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions_exactly():
    for total in (0, 1, 7, 4096, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    assert shard_range(65536, 8, 3) == (3 * 8192, 4 * 8192)


def test_tree_levels():
    assert tree_levels(256) == [128, 64, 32, 16, 8, 4, 2, 1]
    assert sum(tree_levels(256)) == 255


def test_gloo_world2_broadcast_and_gather():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_keys, ok_map, ok_tree in res:
        assert ok_keys, f"rank {rank}: key broadcast mismatch"
        assert ok_map, f"rank {rank}: sharded map/gather mismatch"
        assert ok_tree, f"rank {rank}: tree reduction mismatch"
