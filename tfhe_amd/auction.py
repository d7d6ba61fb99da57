"""Encrypted max-tree (BASELINE.json config C5: "examples/blind-auction FheUint32 comparison tree
(chained PBS + carry), 256 bidders, 8xMI355X"; SURVEY §8d C5: 255 FheUint32 `max` comparisons in 8
dependent levels 128, 64, ..., 1).

Each comparison keeps the larger bid and the bidder index that holds it (ties keep the lower index,
as a first-price auction that accepts the earliest highest bid): one `ge` carry chain, then one
select over the concatenated (bid | index) bits with the shared condition.  All comparisons of a
level run in lockstep on the circuit (one PBS launch per circuit level); with a process group the
level's pairs are sharded over the ranks (one GPU each) and the winners all_gathered
(tfhe_amd.dist.sharded_map) — the only collective, once per tree level.
"""
from __future__ import annotations

import numpy as np

from .integer import Circuit, FheUint, g_ge, g_select


def _level_op(c: Circuit, lhs: np.ndarray, rhs: np.ndarray, w: int):
    """lhs / rhs: (P, w + iw, dim) = (bid bits | index bits); returns the winners (P, w + iw, dim)."""
    ge = yield from g_ge(c, lhs[:, :w], rhs[:, :w])
    return (yield from g_select(ge, lhs, rhs))


def _run_level(c: Circuit, pairs: np.ndarray, w: int) -> np.ndarray:
    if pairs.shape[0] == 0:
        return pairs[:, 0]
    return c.run(_level_op(c, np.ascontiguousarray(pairs[:, 0]), np.ascontiguousarray(pairs[:, 1]), w))


def max_tree(c: Circuit, bids: FheUint, group=None):
    """Returns (max bid: FheUint of width w, winner index: FheUint of width ceil(log2 B)), batch 1."""
    B, w, dim = bids.bits.shape
    iw = max(1, (B - 1).bit_length())
    idx = FheUint.trivial(c, np.arange(B, dtype=np.uint64), iw).bits        # public positions
    cur = np.concatenate([bids.bits, idx], axis=1)                           # (B, w + iw, dim)
    while cur.shape[0] > 1:
        P = cur.shape[0] // 2
        pairs = cur[: 2 * P].reshape(P, 2, w + iw, dim)
        if group is None:
            win = _run_level(c, pairs, w)
        else:
            import torch

            from .dist import sharded_map
            t = torch.from_numpy(pairs.view(np.int64).copy())
            win_t = sharded_map(t, lambda s: torch.from_numpy(
                _run_level(c, s.numpy().view(np.uint64), w).view(np.int64).copy()), group=group)
            win = win_t.numpy().view(np.uint64).reshape(P, w + iw, dim)
        cur = np.concatenate([win, cur[2 * P:]], axis=0)                      # odd leftover advances
    return FheUint(c, cur[:, :w]), FheUint(c, cur[:, w:])
