"""Multi-GPU decomposition of the hot path.

The top-level domain is split into x-slabs, one per rank (one process per
GPU). A rank owns the i-particles of its slab and holds a read-only halo of
every particle within `reach` of the slab (periodic). The density and force
loops of owned particles then need nothing from other ranks: there is no
cross-cell reduction inside a loop (gather formulation), so the loops run
with no collective. Halo particles are marked inactive (time_bin above
max_active_bin), so the loops read them as neighbours and never update them
— the same mechanism SWIFT uses for inactive/foreign cells.
"""
from __future__ import annotations

import numpy as np

from . import abi


def slab_bounds(rank: int, world: int, length: float):
    w = length / world
    return rank * w, (rank + 1) * w


def slab_local_set(parts: np.ndarray, rank: int, world: int, box_x: float, reach: float,
                   halo_time_bin: int = 2):
    """Owned + halo particles of `rank`'s x-slab of a periodic box of length
    box_x. Returns (local AoS array, n_owned): owned particles first (time bins
    unchanged), then halo particles with time_bin = halo_time_bin."""
    lo, hi = slab_bounds(rank, world, box_x)
    x = np.mod(parts["x"][:, 0], box_x)
    owned = (x >= lo) & (x < hi)
    if world == 1:
        out = abi.copy_parts(parts)
        return out, len(parts)
    # periodic distance of x to the slab [lo, hi)
    d_lo = np.mod(lo - x, box_x)  # distance below the slab
    d_hi = np.mod(x - hi, box_x)  # distance above the slab
    halo = (~owned) & ((d_lo <= reach) | (d_hi < reach))
    own_idx = np.nonzero(owned)[0]
    halo_idx = np.nonzero(halo)[0]
    out = abi.new_parts(len(own_idx) + len(halo_idx))
    out[: len(own_idx)] = parts[own_idx]
    out[len(own_idx):] = parts[halo_idx]
    out["time_bin"][len(own_idx):] = halo_time_bin
    return out, len(own_idx)
