"""Config C5 (encrypted max-tree over 256 FheUint32 bids, tfhe_amd/auction.py) on CPU: the circuit
with the cleartext gate-bootstrap double of test_integer.py, single rank and sharded over a gloo
world of 2 (the per-level shard -> all_gather of the multi-GPU path).  The MI355X run is in
tests/test_gpu_configs.py."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from tfhe_amd import integer as I
from tfhe_amd.auction import max_tree
from test_integer import ClearKey, CleartextEngine


def _bids(B, seed=5):
    v = np.random.default_rng(seed).integers(0, 2**32, B, dtype=np.uint64)
    v[B // 3] = v[2 * B // 3] = np.uint64(2**32 - 7)     # a tie at the top: the lower index wins
    v[-1] = np.uint64(2**32 - 8)
    return v


def _expected(v):
    m = int(v.max())
    return m, int(np.nonzero(v == m)[0][0])


def test_max_tree_256_cleartext():
    v = _bids(256)
    c = I.Circuit(CleartextEngine())
    mx, idx = max_tree(c, I.FheUint.trivial(c, v, 32))
    ck = ClearKey()
    assert (int(mx.decrypt(ck)[0]), int(idx.decrypt(ck)[0])) == _expected(v)
    assert idx.width == 8


def test_max_tree_ragged_cleartext():
    v = _bids(37, seed=9)
    c = I.Circuit(CleartextEngine())
    mx, idx = max_tree(c, I.FheUint.trivial(c, v, 32))
    ck = ClearKey()
    assert (int(mx.decrypt(ck)[0]), int(idx.decrypt(ck)[0])) == _expected(v)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        v = _bids(64, seed=11)
        eng = CleartextEngine()
        c = I.Circuit(eng)
        mx, idx = max_tree(c, I.FheUint.trivial(c, v, 32), group=dist.group.WORLD)
        ck = ClearKey()
        q.put((rank, int(mx.decrypt(ck)[0]), int(idx.decrypt(ck)[0]), c.pbs_count))
    finally:
        dist.destroy_process_group()


def test_max_tree_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _expected(_bids(64, seed=11))
    for rank, mx, idx, pbs in res:
        assert (mx, idx) == want, rank
    # the comparisons were split: each rank bootstrapped only part of the tree
    c = I.Circuit(CleartextEngine())
    max_tree(c, I.FheUint.trivial(c, _bids(64, seed=11), 32))
    assert max(r[3] for r in res) < c.pbs_count
