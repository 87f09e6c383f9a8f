"""Edges of the small-leaf batch P2P (p2p_batch_kernel, swh_grav.hip): the
staging of up to 32 consecutive P-P entries into one kPPBatch = 256-gpart LDS
tile.

* A P-P entry whose source holds more gparts than the tile: the no-cache
  entries of runner_dopair_recursive_grav (runner_doiact_grav.c:2297-2302,
  runner_dopair_grav_pp_no_cache 1440-1483) put a single-gpart cell against
  a whole split cell, so the source is a split cell of any size while every
  leaf is small. The batch must hold that entry alone and stage it in chunks.
* Zero-count leaves inside a 32-entry batch (leaf lists over a sparse box):
  an entry that stages nothing must neither end the batch early nor shift
  the gpart -> entry map of the entries after it.

Both are checked against the fp64 oracle (grav_tree / grav_pp_leaves): exact
P2P (and M2P) counts, a_grav and potential to 1e-6 of the largest component.

DESIGN.md §4.2 ("The round-4 grav_tree fault") records the fault these edges
caused in an unreleased round-4 build."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
from swift_subtask_dev_amd import abi, ics

pytestmark = pytest.mark.gpu

K_PP_BATCH = 256  # swh_grav.hip kPPBatch


def _grav_params(periodic=False, theta=0.5, r_cut_max=0.0, r_s_inv=0.0, r_cut_min=0.0):
    G = abi.GravParams(1 if periodic else 0, (C.c_float * 3)(1, 1, 1), r_s_inv, r_cut_min,
                       abi.NUM_TIME_BINS)
    G.theta_crit = theta
    G.adaptive_tolerance = 1e-4
    G.use_advanced_MAC = 0
    G.r_cut_max = r_cut_max
    return G


def _close(g, o, rel=1e-6):
    a, b = g["a_grav"].astype(np.float64), o["a_grav"].astype(np.float64)
    e = np.abs(a - b).max(axis=1)
    if e.max() > rel * np.abs(b).max():
        for k in np.argsort(-e)[:6]:
            print(f"gpart {k}: x {g['x'][k]} gpu {a[k]} oracle {b[k]}")
    assert e.max() <= rel * np.abs(b).max(), e.max() / np.abs(b).max()
    p, q = g["potential"].astype(np.float64), o["potential"].astype(np.float64)
    assert np.abs(p - q).max() <= rel * np.abs(q).max()


def _lonely_cell_box(n_clump=700, seed=11):
    """A clump of n_clump gparts in top cell (0,0,0) of a 2^3 grid, exactly
    one gpart in top cell (1,0,0), a sparse background elsewhere."""
    rng = np.random.Generator(np.random.PCG64(seed))
    bg = ics.uniform_gravity_box(6, epsilon=1e-3, seed=seed)
    x = bg["x"]
    top = np.minimum((np.mod(x, 1.0) / 0.5).astype(int), 1)
    keep = ~((top[:, 1] == 0) & (top[:, 2] == 0))  # cells (0,0,0) and (1,0,0) filled below
    bg = bg[keep]
    n = len(bg) + n_clump + 1
    g = np.zeros(n, dtype=bg.dtype)
    g[: len(bg)] = bg
    tmpl = bg[0]
    g[len(bg):] = tmpl
    clump = np.clip(0.25 + rng.normal(0, 0.06, (n_clump, 3)), 0.01, 0.49)
    g["x"][len(bg): len(bg) + n_clump] = clump
    g["x"][-1] = (0.75, 0.25, 0.25)
    g["id_or_neg_offset"] = np.arange(n)
    return g


@pytest.mark.parametrize("theta,periodic", [(1e-6, False), (0.4, False), (0.4, True)])
def test_tree_no_cache_source_larger_than_tile(gpu_ctx, theta, periodic):
    from swift_subtask_dev_amd import lib
    g0 = _lonely_cell_box()
    g, cells, tops = ics.gravity_tree(g0, 2, split_size=32)
    counts = cells["count"][tops]
    assert sorted(counts)[:1] == [1] and counts.max() > K_PP_BATCH + 200
    leaf = cells["split"] == 0
    assert cells["count"][leaf].max() <= 64  # the small-leaf batch kernel runs
    pairs = ics.top_level_pairs(tops)
    r_s = 1.25 / 16
    G = (_grav_params(True, theta, r_cut_max=10.0, r_s_inv=1 / r_s, r_cut_min=0.1 * r_s)
         if periodic else _grav_params(False, theta))
    gg, go = abi.copy_parts(g), abi.copy_parts(g)
    gs = lib.GravSpace(gpu_ctx)
    gs.upload(gg)
    gs.set_tree(cells)
    st = gs.tree(G, tops, pairs)
    gs.download(gg)
    gs.close()
    so = np.zeros(6, dtype=np.int64)
    ft = np.zeros((len(cells), 35), dtype=np.float32)
    O.fn("f64", "grav_tree")(go.ctypes.data, len(go), cells.ctypes.data, len(cells),
                             tops.ctypes.data, len(tops), pairs.ctypes.data, len(pairs),
                             C.byref(G), so.ctypes.data, ft.ctypes.data)
    assert [st["n_pp"], st["n_m2p"], st["n_m2l"], st["n_pp_tasks"], st["n_skipped"],
            st["n_pp_truncated"]] == list(so)
    # the lonely gpart's no-cache entry took every gpart of the clump's cell
    lonely = int(np.argmin(np.abs(g["x"][:, 0] - 0.75) + np.abs(g["x"][:, 1] - 0.25)
                           + np.abs(g["x"][:, 2] - 0.25)))
    assert np.abs(gg["a_grav"][lonely]).max() > 0
    _close(gg, go, 2e-6)


def _sparse_leaves(reach, periodic, seed=5):
    """A sparse box in an 8^3 leaf grid (most leaves empty): every leaf
    interacts with every leaf within `reach` cells, so each 32-entry batch
    mixes empty and non-empty sources, and empty i-leaves carry lists."""
    gp = ics.uniform_gravity_box(7, epsilon=0.01, seed=seed)  # 343 gparts
    gp["old_a_grav_norm"] = np.random.Generator(np.random.PCG64(seed)).uniform(20, 200, len(gp))
    cdim = 8
    gs, leaves = ics.leaf_cells(gp, cdim)
    offs, js = [0], []
    for cx in range(cdim):
        for cy in range(cdim):
            for cz in range(cdim):
                seen = []
                for dx in range(-reach, reach + 1):
                    for dy in range(-reach, reach + 1):
                        for dz in range(-reach, reach + 1):
                            nx, ny, nz = cx + dx, cy + dy, cz + dz
                            if periodic:
                                nx, ny, nz = nx % cdim, ny % cdim, nz % cdim
                            elif not (0 <= nx < cdim and 0 <= ny < cdim and 0 <= nz < cdim):
                                continue
                            j = (nx * cdim + ny) * cdim + nz
                            if j not in seen:
                                seen.append(j)
                js.extend(seen)
                offs.append(len(js))
    pairs = np.zeros(len(js), dtype=abi.LEAF_PAIR_DTYPE)
    pairs["j"] = js
    return gs, leaves, np.asarray(offs, dtype=np.int32), pairs


@pytest.mark.parametrize("periodic,truncated,mpole", [(False, 0, False), (True, 1, False),
                                                       (False, 0, True), (True, 1, True)])
def test_batch_zero_count_leaves(gpu_ctx, periodic, truncated, mpole):
    from swift_subtask_dev_amd import lib
    gs, leaves, offs, pairs = _sparse_leaves(2, periodic)
    empty = leaves["count"] == 0
    assert empty.mean() > 0.3 and leaves["count"].max() <= 64
    # some batch (32 consecutive entries) holds empty and non-empty sources
    src_empty = empty[pairs["j"]]
    assert any(src_empty[q:q + 32].any() and (~src_empty[q:q + 32]).any()
               for q in range(0, len(pairs), 32))
    pairs["truncated"] = truncated
    if mpole:
        own = pairs["j"] == np.repeat(np.arange(len(leaves)), np.diff(offs))
        pairs["allow_mpole"] = np.where(own, 0, 1)
    G = _grav_params(periodic, 0.9, r_cut_max=10.0,
                     r_s_inv=1.0 / 0.3 if truncated else 0.0,
                     r_cut_min=0.0 if truncated else 1e30)
    g = gs.copy()
    sp = lib.GravSpace(gpu_ctx)
    sp.upload(g)
    sp.set_leaves(leaves, offs, pairs)
    mp = sp.make_multipoles(want=True) if mpole else None
    n, nm = sp.pp(G, m2p=True)
    sp.download(g)
    sp.close()
    o = gs.copy()
    nmo = C.c_longlong(0)
    no = O.fn("f64", "grav_pp_leaves")(o.ctypes.data, leaves.ctypes.data, len(leaves),
                                       offs.ctypes.data, pairs.ctypes.data, C.byref(G),
                                       C.cast(mp, C.c_void_p) if mpole else None,
                                       C.byref(nmo))
    assert n == no and nm == nmo.value, (n, no, nm, nmo.value)
    if mpole:
        assert nm > 0
    _close(g, o)
