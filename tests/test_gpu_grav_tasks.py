"""The recursive gravity tasks with SWIFT's signatures (src/runner_doiact_grav.h:
28-37) through the adapter: runner_doself_recursive_grav on every top cell,
runner_dopair_recursive_grav on every top pair, then runner_do_grav_down on
every top cell -- SWIFT's per-task order -- on SWIFT-layout cells (struct cell
with progeny, struct gravity_tensors read by name). Against the batch
swh_grav_tree on the same tree and the same multipoles: the accelerations,
potentials and pushed-down field tensors agree to float accumulation
(the per-task path adds each task's results into the float gpart fields)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from swift_subtask_dev_amd import abi, ics
from test_gpu_tree import clumpy_box, params

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def adapter():
    from swift_subtask_dev_amd import lib
    ad = lib.load_adapter()
    assert ad.swifthip_swift_init(0, 0) == 0
    yield ad


def _swift_cells(g, cells, mp, ti_current):
    """struct cell + struct gravity_tensors mirrors of the tree."""
    n = len(cells)
    cs = (abi.Cell * n)()
    tens = (abi.GravityTensors * n)()
    base = g.ctypes.data
    stride = g.dtype.itemsize
    act = g["time_bin"] <= abi.NUM_TIME_BINS
    for c in range(n):
        rec = cells[c]
        cc = cs[c]
        cc.loc[:] = tuple(rec["loc"])
        cc.width[:] = tuple(rec["width"])
        cc.split = int(rec["split"])
        cc.nodeID = 0
        for k in range(8):
            p = int(rec["progeny"][k])
            cc.progeny[k] = C.addressof(cs[p]) if p >= 0 else None
        s0, cnt = int(rec["start"]), int(rec["count"])
        cc.grav.parts = base + s0 * stride
        cc.grav.count = cnt
        tens[c].set_from(mp[c])
        cc.grav.multipole = C.pointer(tens[c])
        cc.grav.ti_end_min = ti_current if act[s0:s0 + cnt].any() else ti_current - 1
    return cs, tens


@pytest.mark.parametrize("theta", [0.7, 0.4])
def test_recursive_tasks_equal_batch_tree(gpu_ctx, adapter, theta):
    from swift_subtask_dev_amd import lib
    g, cells, tops = ics.gravity_tree(clumpy_box(12, seed=4), 2, split_size=24)
    pairs = ics.top_level_pairs(tops)
    G = params(theta=theta)
    # the batch: the whole step's tasks in one call, its multipoles kept
    gb = abi.copy_parts(g)
    gs = lib.GravSpace(gpu_ctx)
    gs.upload(gb)
    gs.set_tree(cells)
    st = gs.tree(G, tops, pairs)
    gs.download(gb)
    mp = gs.multipoles()
    fb = gs.field_tensors()
    gs.close()
    assert st["n_m2l"] > 0 and st["n_pp"] > 0

    # the same tasks one by one through SWIFT's signatures
    gt = abi.copy_parts(g)
    cs, tens = _swift_cells(gt, cells, mp, 8)
    gp = abi.GravityProps(0, 0, 0, 1e-4, theta, 0, 0)
    eb = abi.EngineBundle(dim=(1.0, 1.0, 1.0), periodic=False, gravity_props=gp)
    rp = C.addressof(eb.runner)
    adapter.swifthip_swift_clear_error()
    for c in tops:
        adapter.runner_doself_recursive_grav(rp, C.addressof(cs[int(c)]), 0)
    for i, j in np.asarray(pairs).reshape(-1, 2):
        adapter.runner_dopair_recursive_grav(rp, C.addressof(cs[int(i)]), C.addressof(cs[int(j)]), 0)
    assert not adapter.swifthip_swift_last_error()
    # the M2L sums are in the cells' tensors, not yet in the particles
    assert any(tens[c].pot.interacted for c in range(len(cells)))
    for c in tops:
        adapter.runner_do_grav_down(rp, C.addressof(cs[int(c)]), 0)
    err = adapter.swifthip_swift_last_error()
    assert not err, err

    a_t, a_b = gt["a_grav"].astype(np.float64), gb["a_grav"].astype(np.float64)
    scale = np.linalg.norm(a_b, axis=1)
    e = np.linalg.norm(a_t - a_b, axis=1) / np.maximum(scale, 1e-30)
    assert e.max() < 1e-5, (e.max(), int(np.argmax(e)))
    ep = np.abs(gt["potential"] - gb["potential"]) / np.maximum(np.abs(gb["potential"]), 1e-30)
    assert ep.max() < 1e-5, ep.max()
    # pushed-down field tensors of the non-root cells, per order
    ft = np.array([[getattr(tens[c].pot, "F_" + n) for n in abi._TENSOR_NAMES]
                   for c in range(len(cells))], dtype=np.float64)
    inner = np.setdiff1d(np.arange(len(cells)), np.asarray(tops))
    for lo, hi in ((0, 1), (1, 4), (4, 10), (10, 20), (20, 35)):
        s = np.abs(fb[inner, lo:hi]).max()
        if s > 0:
            assert np.abs(ft[inner, lo:hi] - fb[inner, lo:hi]).max() <= 1e-5 * s, (lo, hi)


def test_recursive_tasks_inactive_cells_untouched(gpu_ctx, adapter):
    """A pair task with both cells inactive returns at once (no particle or
    tensor changes), and grav_down leaves inactive particles alone."""
    from swift_subtask_dev_amd import lib
    g, cells, tops = ics.gravity_tree(clumpy_box(10, seed=6), 2, split_size=24)
    gs = lib.GravSpace(gpu_ctx)
    gb = abi.copy_parts(g)
    gs.upload(gb)
    gs.set_tree(cells)
    gs.tree(params(), tops, ics.top_level_pairs(tops))
    mp = gs.multipoles()
    gs.close()
    gt = abi.copy_parts(g)
    cs, tens = _swift_cells(gt, cells, mp, 8)
    for c in range(len(cells)):
        cs[c].grav.ti_end_min = 4  # nothing active at ti_current 8
    eb = abi.EngineBundle(dim=(1.0, 1.0, 1.0), periodic=False)
    rp = C.addressof(eb.runner)
    before = gt.copy()
    adapter.swifthip_swift_clear_error()
    i, j = np.asarray(ics.top_level_pairs(tops)).reshape(-1, 2)[0]
    adapter.runner_dopair_recursive_grav(rp, C.addressof(cs[int(i)]), C.addressof(cs[int(j)]), 0)
    adapter.runner_doself_recursive_grav(rp, C.addressof(cs[int(tops[0])]), 0)
    assert not adapter.swifthip_swift_last_error()
    assert np.array_equal(gt["a_grav"], before["a_grav"])
    assert not any(tens[c].pot.interacted for c in range(len(cells)))
