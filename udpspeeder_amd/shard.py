"""Multi-GPU sharding of FEC groups.

FEC groups are independent, so ranks own disjoint, contiguous group ranges
and never exchange data: no collective sits on the data path.  The only
collectives are the bench's barrier and max-over-ranks of the timed region.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np


def weak_range(rank: int, groups_per_rank: int) -> Tuple[int, int]:
    """Weak scaling: every rank owns groups_per_rank groups."""
    g0 = rank * groups_per_rank
    return g0, g0 + groups_per_rank


def strong_range(rank: int, world: int, total: int) -> Tuple[int, int]:
    """Strong scaling: a fixed total split into contiguous near-equal ranges."""
    return total * rank // world, total * (rank + 1) // world


def balanced_ranges(work: Sequence[int], world: int):
    """Contiguous ranges with near-equal summed work (ragged C3: work = (k+m)*len)."""
    w = np.asarray(work, np.float64)
    c = np.concatenate([[0.0], np.cumsum(w)])
    total = c[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(c, total * r / world)))
    cuts.append(len(w))
    return [(cuts[r], cuts[r + 1]) for r in range(world)]
