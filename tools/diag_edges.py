"""Diagnose test_tree_no_cache_source_larger_than_tile[0.4-True]: the worst
particles of the GPU tree vs the oracle, and GPU run-to-run determinism."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import oracle_lib as O  # noqa: E402
import test_gpu_grav_edges as T  # noqa: E402
from swift_subtask_dev_amd import abi, ics, lib  # noqa: E402

g0 = T._lonely_cell_box()
g, cells, tops = ics.gravity_tree(g0, 2, split_size=32)
pairs = ics.top_level_pairs(tops)
r_s = 1.25 / 16
G = T._grav_params(True, 0.4, r_cut_max=10.0, r_s_inv=1 / r_s, r_cut_min=0.1 * r_s)
ctx = lib.Context(0, "f64")
res = []
for rep in range(3):
    gg = abi.copy_parts(g)
    gs = lib.GravSpace(ctx)
    gs.upload(gg)
    gs.set_tree(cells)
    st = gs.tree(G, tops, pairs)
    gs.download(gg)
    gs.close()
    res.append((gg, st))
go = abi.copy_parts(g)
so = np.zeros(6, dtype=np.int64)
O.fn("f64", "grav_tree")(go.ctypes.data, len(go), cells.ctypes.data, len(cells), tops.ctypes.data,
                         len(tops), pairs.ctypes.data, len(pairs), C.byref(G), so.ctypes.data, None)
print("oracle stats", list(so))
leaf_of = np.full(len(g), -1)
for c in range(len(cells)):
    if not cells["split"][c]:
        leaf_of[cells["start"][c]:cells["start"][c] + cells["count"][c]] = c
for rep, (gg, st) in enumerate(res):
    e = np.abs(gg["a_grav"].astype(np.float64) - go["a_grav"]).max(axis=1)
    worst = np.argsort(-e)[:8]
    print(f"rep {rep}: stats {st['n_pp'], st['n_m2p'], st['n_m2l'], st['n_pp_tasks'], st['n_skipped']} max err {e.max():.3e}")
    for k in worst:
        c = leaf_of[k]
        print(f"   gpart {k} leaf {c} (count {cells['count'][c]}) x {g['x'][k]} err {e[k]:.3e} |a| {np.abs(go['a_grav'][k]).max():.3e}")
print("reps bitwise equal:", all(np.array_equal(res[0][0]["a_grav"], r[0]["a_grav"]) for r in res))
