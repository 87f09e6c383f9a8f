"""The M-M gravity tasks outside the recursive walk, with SWIFT's signatures
(src/runner_doiact_grav.h:39-43), through the adapter on SWIFT-layout cells:

* runner_dopair_grav_mm_progenies (runner_doiact_grav.c:2067-2093): the
  progeny pairs whose bit 8 i + j is set in the task flags get
  runner_dopair_grav_mm -- symmetric M2L when both progenies are active and
  local, else the active one receives (nonsym);
* runner_do_grav_long_range (2441-2530): a cell against every top-level cell
  with particles except its own top cell: skipped beyond r_cut_max (periodic,
  cell_min_dist2_same_size), M2L from the top cell when cell_can_use_pair_mm
  accepts on the rebuild data.

Both against the f64 oracle's M2L of the same pairs (grav_m2l_pairs, the
tree walk's M2L restated) with the pair sets derived independently here from
the reference's rules and the oracle's MAC; the GPU's field tensors are added
into c->grav.multipole->pot (interacted = 1 on the targets only)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
from swift_subtask_dev_amd import abi, ics
from test_gpu_grav_tasks import _swift_cells
from test_gpu_tree import clumpy_box

pytestmark = pytest.mark.gpu

TI = 8


@pytest.fixture(scope="module")
def adapter():
    from swift_subtask_dev_amd import lib
    ad = lib.load_adapter()
    assert ad.swifthip_swift_init(0, 0) == 0
    yield ad


def _tree(gpu_ctx, ntop, seed, periodic):
    """A split cell tree with the library's multipoles (rebuild data = current)."""
    from swift_subtask_dev_amd import lib
    g, cells, tops = ics.gravity_tree(clumpy_box(12, seed=seed), ntop, split_size=24)
    gs = lib.GravSpace(gpu_ctx)
    gs.upload(abi.copy_parts(g))
    gs.set_tree(cells)
    G0 = abi.GravParams(1 if periodic else 0, (C.c_float * 3)(1, 1, 1), 0.0, 0.0,
                        abi.NUM_TIME_BINS)
    G0.theta_crit = 0.5
    gs.tree(G0, tops, ics.top_level_pairs(tops))
    mp = gs.multipoles()
    gs.close()
    gt = abi.copy_parts(g)
    cs, tens = _swift_cells(gt, cells, mp, TI)
    for c in range(len(cells)):
        tens[c].CoM_rebuild[:] = tuple(tens[c].CoM)
        tens[c].r_max_rebuild = tens[c].r_max
        cs[c].grav.ti_old_multipole = TI
        cs[c].grav.ti_end_min = TI
        for k in range(8):
            p = int(cells[c]["progeny"][k])
            if p >= 0:
                cs[p].parent = C.addressof(cs[c])
    return g, cells, tops, mp, cs, tens


def _pot(tens, c):
    return np.array([getattr(tens[c].pot, "F_" + n) for n in abi._TENSOR_NAMES], dtype=np.float64)


def _check(tens, want, targets, ncells):
    """GPU tensors vs the oracle's, per multipole order (fp64 vs fp64: the
    float field tensors' rounding)."""
    got = np.stack([_pot(tens, c) for c in range(ncells)])
    for lo, hi in ((0, 1), (1, 4), (4, 10), (10, 20), (20, 35)):
        s = np.abs(want[:, lo:hi]).max()
        if s > 0:
            d = np.abs(got[:, lo:hi] - want[:, lo:hi]).max()
            assert d <= 2e-6 * s, (lo, hi, d / s)
    for c in range(ncells):
        assert bool(tens[c].pot.interacted) == (c in targets), c


def _grav_params(periodic, theta, r_s_inv=0.0, r_cut_max=0.0):
    G = abi.GravParams(1 if periodic else 0, (C.c_float * 3)(1, 1, 1), r_s_inv, 0.0, 0)
    G.theta_crit = theta
    G.r_cut_max = r_cut_max
    return G


@pytest.mark.parametrize("inactive", [False, True])
def test_mm_progenies_vs_oracle(gpu_ctx, adapter, inactive):
    g, cells, tops, mp, cs, tens = _tree(gpu_ctx, 2, seed=13, periodic=False)
    split = [int(t) for t in tops if cells["split"][int(t)]]
    assert len(split) >= 2
    ci, cj = split[0], split[-1]
    prog_i = [int(p) for p in cells["progeny"][ci]]
    prog_j = [int(p) for p in cells["progeny"][cj]]
    rng = np.random.Generator(np.random.PCG64(5))
    if inactive:  # some progenies inactive: those pairs are nonsym or skipped
        for p in prog_i[::3] + prog_j[1::3]:
            if p >= 0:
                cs[p].grav.ti_end_min = TI - 1
    flags = 0
    pairs = []
    for i in range(8):
        for j in range(8):
            if prog_i[i] < 0 or prog_j[j] < 0 or rng.random() < 0.3:
                continue
            flags |= 1 << (i * 8 + j)
            a, b = prog_i[i], prog_j[j]
            da, db = cs[a].grav.ti_end_min == TI, cs[b].grav.ti_end_min == TI
            if da and db:
                pairs += [(a, b, 1), (b, a, 1)]
            elif da:
                pairs.append((a, b, 0))
            elif db:
                pairs.append((b, a, 0))
    assert pairs
    gp = abi.GravityProps(0, 0, 0, 1e-4, 0.5, 0, 0)
    eb = abi.EngineBundle(dim=(1.0, 1.0, 1.0), periodic=False, gravity_props=gp,
                          ti_current=TI)
    adapter.swifthip_swift_clear_error()
    adapter.runner_dopair_grav_mm_progenies(C.addressof(eb.runner), C.c_longlong(flags),
                                            C.addressof(cs[ci]), C.addressof(cs[cj]))
    err = adapter.swifthip_swift_last_error()
    assert not err, err
    G = _grav_params(False, 0.5)
    want = np.zeros((len(cells), 35))
    pa = np.asarray(pairs, dtype=np.int32).ravel()
    O.fn("f64", "grav_m2l_pairs")(C.byref(G), mp, len(cells), pa.ctypes.data, len(pairs),
                                  want.ctypes.data)
    print(f"\nmm_progenies: {len(pairs)} directed M2L, "
          f"{sum(1 for p in pairs if p[2])} symmetric")
    _check(tens, want, {p[0] for p in pairs}, len(cells))


@pytest.mark.parametrize("periodic", [False, True])
def test_long_range_vs_oracle(gpu_ctx, adapter, periodic):
    g, cells, tops, mp, cs, tens = _tree(gpu_ctx, 4, seed=17, periodic=periodic)
    # 4^3 top cells of width 0.25: gaps 0.25 (one cell between along an axis)
    # stay within r_cut_max = 0.3, diagonal gaps (0.35, 0.43) are skipped
    r_s = 0.3 / 4.5
    r_cut_max = 4.5 * r_s if periodic else 0.0
    theta = 0.95
    tops_i = np.asarray(tops, dtype=np.int32)
    with_parts = np.ascontiguousarray(tops_i[cells["count"][tops_i] > 0])
    mesh = abi.PmMesh(1 if periodic else 0, (C.c_double * 3)(1, 1, 1),
                      1.0 / r_s if periodic else 0.0, 0.0, r_cut_max)
    gp = abi.GravityProps(0, 0, 0, 1e-4, theta, 0, 0)
    eb = abi.EngineBundle(dim=(1.0, 1.0, 1.0), periodic=periodic, gravity_props=gp, mesh=mesh,
                          ti_current=TI)
    eb.space.cells_top = C.addressof(cs[0])  # cells_top[k] = cs[k]: the top indices address cs
    eb.space.cells_with_particles_top = with_parts.ctypes.data_as(C.POINTER(C.c_int))
    eb.space.nr_cells_with_particles = len(with_parts)
    G = _grav_params(periodic, theta, 1.0 / r_s if periodic else 0.0, r_cut_max)
    # the task on a top cell and on a sub-cell of another top cell
    top_i = int(tops_i[0])
    sub = next(int(p) for p in cells["progeny"][int(tops_i[5])] if p >= 0)
    targets, pairs, skipped = set(), [], 0
    for ci in (top_i, sub):
        top = ci if ci in set(tops_i.tolist()) else int(tops_i[5])
        for cj in with_parts:
            cj = int(cj)
            if cj == top or mp[cj].M[0] == 0.0:
                continue
            if periodic:
                d2 = 0.0
                for k in range(3):
                    a0, a1 = cells["loc"][top][k], cells["loc"][top][k] + cells["width"][top][k]
                    b0, b1 = cells["loc"][cj][k], cells["loc"][cj][k] + cells["width"][cj][k]
                    near = lambda d: d - 1.0 if d > 0.5 else (d + 1.0 if d < -0.5 else d)  # noqa
                    d2 += min(abs(near(a0 - b0)), abs(near(a0 - b1)), abs(near(a1 - b0)),
                              abs(near(a1 - b1))) ** 2
                if d2 > r_cut_max ** 2:
                    targets.add(ci)
                    skipped += 1
                    continue
            dx = np.array(mp[top].CoM) - np.array(mp[cj].CoM)
            if periodic:
                dx = dx - np.round(dx)
            if O.fn("f64", "grav_m2l_accept_symmetric")(C.byref(G), C.byref(mp[top]),
                                                      C.byref(mp[cj]), float(dx @ dx)):
                pairs.append((ci, cj, 0))
                targets.add(ci)
    assert pairs and (skipped > 0 or not periodic)
    adapter.swifthip_swift_clear_error()
    for ci in (top_i, sub):
        adapter.runner_do_grav_long_range(C.addressof(eb.runner), C.addressof(cs[ci]), 1)
    err = adapter.swifthip_swift_last_error()
    assert not err, err
    want = np.zeros((len(cells), 35))
    pa = np.asarray(pairs, dtype=np.int32).ravel()
    O.fn("f64", "grav_m2l_pairs")(C.byref(G), mp, len(cells), pa.ctypes.data, len(pairs),
                                  want.ctypes.data)
    print(f"\nlong range: {len(pairs)} M2L from {len(with_parts)} top cells, {skipped} beyond "
          f"r_cut_max")
    _check(tens, want, targets, len(cells))


def test_long_range_undrifted_multipole_refused(gpu_ctx, adapter):
    """Outside SWIFT there is no cell_drift_multipole: an undrifted multipole
    is refused (SWIFT's build drifts it, as the reference's task does)."""
    g, cells, tops, mp, cs, tens = _tree(gpu_ctx, 2, seed=3, periodic=False)
    t = int(tops[0])
    cs[t].grav.ti_old_multipole = TI - 2
    eb = abi.EngineBundle(dim=(1.0, 1.0, 1.0), periodic=False, ti_current=TI)
    adapter.swifthip_swift_clear_error()
    adapter.runner_do_grav_long_range(C.addressof(eb.runner), C.addressof(cs[t]), 1)
    assert b"Undrifted multipole" in adapter.swifthip_swift_last_error()
    adapter.swifthip_swift_clear_error()
