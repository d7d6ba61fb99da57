"""Encrypted max-tree (BASELINE.json config C5: "examples/blind-auction FheUint32 comparison tree
(chained PBS + carry), 256 bidders, 8xMI355X"; SURVEY §8d C5: 255 FheUint32 `max` comparisons in 8
dependent levels 128, 64, ..., 1).

Each comparison keeps the larger bid and the bidder index that holds it (ties keep the lower index,
as a first-price auction that accepts the earliest highest bid): one `ge` carry chain, then one
select over the concatenated (bid | index) bits with the shared condition.  All comparisons of a
level run in lockstep on the circuit (one PBS launch per circuit level); with a process group the
level's pairs are sharded over the ranks (one GPU each, a contiguous slice per rank) and the winners
all_gathered (tfhe_amd.dist.sharded_map) — the only collective, once per tree level.  A device-resident
circuit (Circuit(device=...)) keeps the level on the GPU: slice, launch and gather are device tensors (RCCL
all_gather over xGMI under "nccl"; staged through host memory under gloo).

The bidder positions are public, so an index bit stays a clear value while both sides of every pair agree
on it and needs no bootstrap when they differ: ge ? 1 : 0 is the condition itself, ge ? 0 : 1 its negation
(free).  Only index bits that are already encrypted on some candidate go through the select's two PBS.  In
the power-of-two tree, level l therefore selects l encrypted index bits instead of all ceil(log2 B): the
256-bidder tree bootstraps 3,586 fewer ciphertexts (the first level's select launch 10,240 -> 8,192).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from .integer import NOT, Circuit, FheUint, _cat, _contig, _is_t, _stack, _where, g_ge, g_select

# an index bit column over the current candidates: ("pub", bool values (m,)) or ("enc", ciphertexts (m, dim))
Col = Tuple[str, np.ndarray]


def _level_op(c: Circuit, lhs: np.ndarray, rhs: np.ndarray, w: int):
    """lhs / rhs: (P, w + k, dim) = (bid bits | encrypted index bits); returns (P, w + k + 1, dim): the winners'
    selected columns, then the condition ge = lhs >= rhs."""
    ge = yield from g_ge(c, lhs[:, :w], rhs[:, :w])
    sel = yield from g_select(ge, lhs, rhs)
    return _cat([sel, ge[:, None]], axis=1)


def _run_level(c: Circuit, pairs: np.ndarray, w: int) -> np.ndarray:
    if pairs.shape[0] == 0:
        return c.trivial(np.zeros((0, pairs.shape[2] + 1), dtype=bool))
    return c.run(_level_op(c, _contig(pairs[:, 0]), _contig(pairs[:, 1]), w))


def _index_level(c: Circuit, cols: List[Col], enc_sel: np.ndarray, ge: np.ndarray, P: int) -> List[Col]:
    """The winners' index columns: encrypted columns come out of the select (enc_sel, in column order), public
    columns stay public where every pair agrees, else become ge / NOT(ge) / trivial per pair (no PBS).  The
    leftover candidate of an odd level (position 2P) keeps its bit."""
    out, e = [], 0
    for kind, v in cols:
        if kind == "enc":
            out.append(("enc", _cat([enc_sel[:, e], v[2 * P:]], axis=0)))
            e += 1
            continue
        vl, vr = v[0:2 * P:2], v[1:2 * P:2]
        if np.array_equal(vl, vr):
            out.append(("pub", np.concatenate([vl, v[2 * P:]])))
            continue
        triv = c.trivial(vl)
        col = _where((vl & ~vr)[:, None], ge, _where((~vl & vr)[:, None], NOT(ge), triv))
        out.append(("enc", _cat([col, c.trivial(v[2 * P:])], axis=0)))
    return out


def max_tree(c: Circuit, bids: FheUint, group=None):
    """Returns (max bid: FheUint of width w, winner index: FheUint of width ceil(log2 B)), batch 1."""
    B, w, dim = bids.bits.shape
    iw = max(1, (B - 1).bit_length())
    pos = np.arange(B, dtype=np.int64)
    cols: List[Col] = [("pub", ((pos >> j) & 1).astype(bool)) for j in range(iw)]   # public positions
    cur = bids.bits                                                                    # (m, w, dim)
    while cur.shape[0] > 1:
        m = cur.shape[0]
        P = m // 2
        enc = [v for kind, v in cols if kind == "enc"]
        full = _cat([cur] + [v[:, None] for v in enc], axis=1) if enc else cur   # (m, w + k, dim)
        pairs = full[: 2 * P].reshape(P, 2, full.shape[1], dim)
        if group is None:
            res = _run_level(c, pairs, w)
        elif _is_t(pairs):   # device-resident circuit: the level's tensors are sliced and gathered on the device
            from .dist import sharded_map
            res = sharded_map(pairs, lambda s: _run_level(c, s, w), group=group)
        else:
            import torch

            from .dist import sharded_map
            t = torch.from_numpy(pairs.view(np.int64).copy())
            res_t = sharded_map(t, lambda s: torch.from_numpy(
                _run_level(c, s.numpy().view(np.uint64), w).view(np.int64).copy()), group=group)
            res = res_t.cpu().numpy().view(np.uint64).reshape(P, full.shape[1] + 1, dim)
        win, ge = res[:, :-1], res[:, -1]
        cols = _index_level(c, cols, win[:, w:], ge, P)
        cur = _cat([win[:, :w], cur[2 * P:]], axis=0)                          # odd leftover advances
    idx = _stack([v[0] if kind == "enc" else c.trivial(v[:1])[0] for kind, v in cols], axis=0)[None]
    return FheUint(c, cur[:, :w]), FheUint(c, idx)
