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
from test_integer import ClearKey, CleartextEngine, CleartextTorchEngine


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


def test_max_tree_sizes_public_index_bits():
    """Odd leftovers and every tree shape: public index bits turn into encrypted ones (ge / NOT ge / trivial)
    exactly where the pairs disagree, and the winner index is right for every bidder count."""
    for B in (1, 2, 3, 5, 6, 17, 64, 100):
        for seed in (1, 2):
            v = np.random.default_rng(B * 10 + seed).integers(0, 16, B, dtype=np.uint64)   # many ties
            c = I.Circuit(CleartextEngine())
            mx, idx = max_tree(c, I.FheUint.trivial(c, v, 4))
            ck = ClearKey()
            assert (int(mx.decrypt(ck)[0]), int(idx.decrypt(ck)[0])) == _expected(v), (B, seed)


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
        ck = ClearKey()
        out = [rank]
        # host arrays, then the device-resident circuit (torch tensors: sliced and gathered as tensors)
        for dev in (None, "cpu"):
            c = I.Circuit(CleartextTorchEngine(), device=dev)
            mx, idx = max_tree(c, I.FheUint.trivial(c, v, 32), group=dist.group.WORLD)
            out += [int(mx.decrypt(ck)[0]), int(idx.decrypt(ck)[0]), c.pbs_count, type(mx.bits).__name__]
        q.put(tuple(out))
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
    c = I.Circuit(CleartextEngine())
    max_tree(c, I.FheUint.trivial(c, _bids(64, seed=11), 32))
    for rank, mx, idx, pbs, kind, mx_d, idx_d, pbs_d, kind_d in res:
        assert (mx, idx) == want and (mx_d, idx_d) == want, rank
        assert kind == "ndarray" and kind_d == "Tensor"
        # the comparisons were split: each rank bootstrapped only part of the tree, in both circuit forms
        assert pbs == pbs_d and pbs < c.pbs_count
    assert sum(r[3] for r in res) == c.pbs_count


def test_max_tree_launch_shape():
    """The comparisons' carry-out runs as a block ripple + reduction tree sized by the circuit's cost
    model (tfhe_amd.integer._carry_out), and the select is one level (its OR of exclusive terms is linear):
    61 launches for the 256-bidder tree instead of the ripple's 116 (level 1: 8 chain steps of 896 PBS + 2
    tree levels instead of 32 steps of 128, then one select launch).  The bidder positions are public, so level l
    selects only the l index bits already encrypted: the first select launch is 2 x 128 x 32 (bids only) instead of
    2 x 128 x 40, and the tree bootstraps 3,586 ciphertexts fewer (38,168 -> 34,582)."""
    c = I.Circuit(CleartextEngine())
    sizes = []
    pbs = c.engine.pbs
    c.engine.pbs = lambda x, lut, *a, **k: (sizes.append(x.shape[0]), pbs(x, lut, *a, **k))[1]
    v = _bids(256)
    mx, idx = max_tree(c, I.FheUint.trivial(c, v, 32))
    assert (int(mx.decrypt(ClearKey())[0]), int(idx.decrypt(ClearKey())[0])) == _expected(v)
    assert c.launches == len(sizes) == 61
    assert sizes[:11] == [896] * 8 + [384, 128, 8192]
    assert c.pbs_count == sum(sizes) == 38_168 - 3_586
    assert [c.carry_block(B, 32) for B in (128, 64, 32, 1)] == [8, 4, 2, 2]


def test_carry_out_every_block_size():
    """_carry_out at every block size (ragged last blocks included) equals a >= b on random and edge operands."""
    rng = np.random.default_rng(11)
    for w in (1, 5, 8, 13, 32):
        a = rng.integers(0, 1 << w, 40, dtype=np.uint64)
        b = rng.integers(0, 1 << w, 40, dtype=np.uint64)
        b[:6] = a[:6]
        a[6], b[6] = 0, (1 << w) - 1
        a[7], b[7] = (1 << w) - 1, 0
        for s in range(1, w + 1):
            c = I.Circuit(CleartextEngine())
            A, Bv = I.FheUint.trivial(c, a, w).bits, I.FheUint.trivial(c, b, w).bits
            cout = c.run(I._carry_out(c, A, I.NOT(Bv), True, s))
            assert np.array_equal(ClearKey().decrypt_bool(cout), a >= b), (w, s)
            assert c.launches == len(I._carry_levels(40, w, s))
