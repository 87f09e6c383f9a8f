"""GPU drift: swh_space_drift vs the oracle's box_drift
(drift_part, src/drift.h:143-232, with SPHENIX hydro_predict_extra,
src/hydro/SPHENIX/hydro.h:1012-1066), and the loops after a drift without a
rebuild (particles left in their cells, reach widened by dx_max) vs the fp64
oracle chain on the drifted particles: identical interaction counts and the
same tolerances as the rebuilt chain (tests/test_gpu_parity.py).

Float tolerances: the drift is a handful of float operations per field; the
GPU contracts a*b+c into fma where the gcc-built oracle rounds twice, so
fields agree to a few float ulps (x to a few double ulps), not bit for bit.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
from test_gpu_parity import VARIANTS, assert_close, box_chain_oracle
from swift_subtask_dev_amd import abi, ics

pytestmark = pytest.mark.gpu


def _stepped_state(ctx, periodic=True, n=16, seed=5):
    """A box after one full chain: a_hydro, u_dt, h_dt, v_sig are live."""
    from swift_subtask_dev_amd import lib
    P = abi.default_hydro_params(periodic=periodic)
    parts = ics.sedov_box(n, velocity="divergent", pert=0.3, seed=seed)
    sp = lib.HydroSpace(ctx)
    sp.upload(parts)
    sp.rebuild(P)
    sp.hydro_step(P)
    sp.download(parts, abi.FIELDS_ALL)
    sp.close()
    return parts, P


def _xparts(parts, vmax, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    n = len(parts)
    xp = abi.new_xparts(n)
    xp["v_full"] = parts["v"] + rng.uniform(-vmax, vmax, (n, 3)).astype(np.float32)
    xp["a_grav"] = rng.normal(0, 3.0, (n, 3)).astype(np.float32)
    parts["gpart"] = np.where(rng.uniform(size=n) < 0.5, 1, 0).astype(np.uint64)
    return xp


def _drift_params(dt, min_u=0.0):
    return abi.DriftParams(dt, 0.5 * dt, 0.7 * dt, 0.9 * dt, min_u)


def _oracle_drift(parts, xp, D):
    o = abi.copy_parts(parts)
    ox = xp.copy()
    hasg = np.ascontiguousarray((parts["gpart"] != 0).astype(np.int8))
    O.fn("f64", "box_drift")(o.ctypes.data, ox.ctypes.data, hasg.ctypes.data, len(o),
                             C.byref(D))
    return o, ox


@pytest.fixture(scope="module")
def stepped(gpu_ctx):
    return _stepped_state(gpu_ctx)


@pytest.mark.parametrize("min_u", [0.0, 0.3])
def test_drift_vs_oracle(gpu_ctx, stepped, min_u):
    from swift_subtask_dev_amd import lib
    parts0, P = stepped
    parts = abi.copy_parts(parts0)
    xp = _xparts(parts, 0.5, seed=2)
    # some particles cool below min_u, some drift with |w1| >= 0.2 (expf branch)
    parts["u_dt"][::7] = -50.0 * parts["u"][::7]
    parts["h_dt"][::11] *= 40.0
    parts["time_bin"][::13] = abi.TIME_BIN_INHIBITED
    D = _drift_params(0.01, min_u)
    sp = lib.HydroSpace(gpu_ctx)
    g = abi.copy_parts(parts)
    sp.upload(g)
    sp.rebuild(P)
    assert sp.info()["dx_max"] == 0.0
    sp.upload_xparts(xp)
    sp.drift(D, P)
    sp.download(g, abi.FIELDS_DRIFT)
    info = sp.info()
    sp.close()
    o, ox = _oracle_drift(parts, xp, D)
    live = parts["time_bin"] != abi.TIME_BIN_INHIBITED
    assert np.array_equal(g["x"][~live], parts["x"][~live])
    assert np.abs(g["x"] - o["x"]).max() <= 4e-16 * 2
    for f in ("v", "u", "h", "rho", "pressure", "soundspeed", "v_sig"):
        assert_close(g[f], o[f], 1e-6, 1e-7, f)
    assert (g["u"][live] >= min_u).all()
    # dx_max: the largest |x_diff| of the drift (SWIFT's dx_max_part), rounded up
    dref = np.sqrt((ox["x_diff"][live].astype(np.float64) ** 2).sum(axis=1)).max()
    assert dref <= info["dx_max"] <= dref * (1 + 1e-5)
    assert not info["list_valid"]


def test_tuning_rejects_removed_variants(gpu_ctx):
    """Loop variants 1, 4 and 5 (round 1's tile loops) are gone: the pair
    lists are the only loop."""
    from swift_subtask_dev_amd import lib
    sp = lib.HydroSpace(gpu_ctx)
    for v in (1, 4, 5):
        with pytest.raises(lib.SwhError):
            sp.set_tuning(1, v)
    with pytest.raises(lib.SwhError):
        sp.set_tuning(1, 7, 32)
    sp.set_tuning(1, 7, 16, list_keep=1, list_skin=0.2)
    sp.close()


def test_drift_requires_xparts(gpu_ctx, stepped):
    from swift_subtask_dev_amd import lib
    parts, P = stepped
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(abi.copy_parts(parts))
    sp.rebuild(P)
    with pytest.raises(lib.SwhError, match="upload_xparts"):
        sp.drift(_drift_params(0.01), P)
    sp.close()


def _drifted_chain(ctx, parts, xp, Ds, P, variant, **tuning):
    """GPU: rebuild once, drift len(Ds) times, full chain without a rebuild."""
    from swift_subtask_dev_amd import lib
    g = abi.copy_parts(parts)
    sp = lib.HydroSpace(ctx)
    sp.set_tuning(1, variant, 0, **tuning)
    sp.upload(g)
    sp.rebuild(P)
    sp.upload_xparts(xp)
    for D in Ds:
        sp.drift(D, P)
    dx = sp.info()["dx_max"]
    res = sp.hydro_step(P)
    sp.download(g, abi.FIELDS_ALL)
    sp.close()
    return g, res, dx


def _check_chain(g, rg, o, ro):
    assert rg["density"] == ro["density"]
    assert rg["force"] == ro["force"]
    assert_close(g["h"], o["h"], 1e-6, what="h")
    for f in ("rho", "pressure", "soundspeed", "balsara", "v_sig", "laplace_u"):
        assert_close(g[f], o[f], 5e-5, 1e-4, f)
    assert_close(g["a_hydro"], o["a_hydro"], 5e-5, 1e-4, "a_hydro")
    assert_close(g["u_dt"], o["u_dt"], 5e-5, 1e-4, "u_dt")
    assert_close(g["h_dt"], o["h_dt"], 5e-5, 1e-4, "h_dt")
    assert np.array_equal(g["min_ngb_time_bin"], o["min_ngb_time_bin"])


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("periodic", [True, False])
def test_loops_after_drift_vs_f64(gpu_ctx, variant, periodic):
    """Displacements up to ~half a smoothing length; particles cross the
    periodic faces and leave their cells."""
    parts, P = _stepped_state(gpu_ctx, periodic=periodic, n=14, seed=8)
    xp = _xparts(parts, 1.0, seed=3)
    D = _drift_params(0.02)
    g, rg, dx = _drifted_chain(gpu_ctx, parts, xp, [D], P, variant)
    o, _ = _oracle_drift(parts, xp, D)
    assert dx > 0.3 * float(parts["h"].mean())
    if periodic:
        crossed = ((o["x"] < 0) | (o["x"] >= 1.0)).any(axis=1)
        assert crossed.sum() > 10
    o, ro = box_chain_oracle(o, P)
    _check_chain(g, rg, o, ro)


@pytest.mark.parametrize("variant", [7])
def test_repeated_drifts_accumulate_reach(gpu_ctx, variant):
    """Three drifts without a rebuild: dx_max accumulates (x_diff is relative
    to the rebuild), the loops stay exact; a rebuild resets it."""
    from swift_subtask_dev_amd import lib
    parts, P = _stepped_state(gpu_ctx, n=14, seed=9)
    xp = _xparts(parts, 1.0, seed=4)
    Ds = [_drift_params(0.006) for _ in range(3)]
    g, rg, dx = _drifted_chain(gpu_ctx, parts, xp, Ds, P, variant)
    o = parts
    for D in Ds:
        o, _ = _oracle_drift(o, xp, D)
    o, ro = box_chain_oracle(o, P)
    _check_chain(g, rg, o, ro)
    # single-drift reach of the same total displacement, within rounding
    _, _, dx1 = _drifted_chain(gpu_ctx, parts, xp, [_drift_params(0.018)], P, variant)
    assert abs(dx - dx1) <= 1e-5 * dx1
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(abi.copy_parts(parts))
    sp.rebuild(P)
    sp.upload_xparts(xp)
    sp.drift(Ds[0], P)
    assert sp.info()["dx_max"] > 0
    sp.rebuild(P)
    assert sp.info()["dx_max"] == 0.0
    sp.close()


def test_drift_list_skin_and_capacity(gpu_ctx):
    """Pair lists after a drift with a list skin and a small list capacity
    (overflow path) stay exact."""
    parts, P = _stepped_state(gpu_ctx, n=14, seed=10)
    xp = _xparts(parts, 1.0, seed=5)
    D = _drift_params(0.01)
    o, _ = _oracle_drift(parts, xp, D)
    o, ro = box_chain_oracle(o, P)
    for tuning in ({"list_skin": 0.2}, {"list_capacity": 24}):
        g, rg, _ = _drifted_chain(gpu_ctx, parts, xp, [D], P, 7, **tuning)
        _check_chain(g, rg, o, ro)


def test_clustered_adaptive_drift_chain_vs_f64(gpu_ctx):
    """Adaptive grid (clustered box: cells sized by the typical H, per-cell
    reach pruning) after a drift without a rebuild: the per-cell maximum
    reach must follow the cell whose sorted range holds a particle, not the
    cell its drifted position falls in, or force pairs with r < H_j of a
    particle that crossed a face are lost. Counts exact, chain tolerances."""
    from swift_subtask_dev_amd import lib
    P = abi.default_hydro_params()
    parts = ics.clustered_box(16, n_clumps=4, per_clump=1500, seed=23)
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(parts)
    sp.rebuild(P)
    sp.hydro_step(P)
    sp.download(parts, abi.FIELDS_ALL)
    sp.close()
    assert parts["h"].max() / parts["h"].min() > 8
    rng = np.random.Generator(np.random.PCG64(29))
    xp = abi.new_xparts(len(parts))
    xp["v_full"] = rng.normal(0.0, 1.0, (len(parts), 3)).astype(np.float32)
    # move the particles by ~0.4 of the median h: many cross the small cells
    dt = 0.4 * float(np.median(parts["h"]))
    D = abi.DriftParams(dt, 0.0, 0.0, 0.0, 0.0)
    g, rg, dx = _drifted_chain(gpu_ctx, parts, xp, [D], P, 7)
    o, _ = _oracle_drift(parts, xp, D)
    o, ro = box_chain_oracle(o, P)
    # the pair sets are exact; the small random velocities make div_v (and so
    # the Balsara switch) a cancelling sum, compared as test_clustered_box_chain
    assert rg["density"] == ro["density"]
    assert rg["gradient"] == ro["gradient"]
    assert rg["force"] == ro["force"]
    assert_close(g["h"], o["h"], 1e-6, what="h")
    assert_close(g["rho"], o["rho"], 5e-5, 1e-4, "rho")
    assert_close(g["a_hydro"], o["a_hydro"], 1e-4, 1e-3, "a_hydro")
    assert_close(g["u_dt"], o["u_dt"], 1e-4, 1e-3, "u_dt")
    assert np.array_equal(g["min_ngb_time_bin"], o["min_ngb_time_bin"])


@pytest.mark.parametrize("disp,expect_rebuilds", [(0.01, False), (0.25, True)])
def test_kept_lists_across_drifts_vs_f64(gpu_ctx, disp, expect_rebuilds):
    """list_keep: pair lists survive drifts while their skin covers the
    displacement (SWIFT keeps its sorts until dx_max_sort exceeds
    space_maxreldx, space.h:66) and the device rebuilds them as soon as some
    H + 2 D exceeds a build reach. Three drifts, each followed by the force
    loop (r < max(H_i, H_j), the widest criterion) on the drifted state vs
    the fp64 oracle; then a density loop on the kept lists. Exact counts and
    the loop tolerances either way; small moves keep the lists (one build),
    large ones force device-side rebuilds."""
    from swift_subtask_dev_amd import lib
    parts, P = _stepped_state(gpu_ctx, n=14, seed=12)
    rng = np.random.Generator(np.random.PCG64(3))
    xp = abi.new_xparts(len(parts))
    xp["v_full"] = rng.normal(0.0, 0.577, (len(parts), 3)).astype(np.float32)
    vmax = float(np.sqrt((xp["v_full"].astype(np.float64) ** 2).sum(axis=1)).max())
    D = abi.DriftParams(disp * float(np.median(parts["h"])) / vmax, 0.0, 0.0, 0.0, 0.0)
    sp = lib.HydroSpace(gpu_ctx)
    sp.set_tuning(1, 0, 0, list_skin=0.2, list_keep=1)
    sp.upload(abi.copy_parts(parts))
    sp.rebuild(P)
    sp.upload_xparts(xp)
    o = abi.copy_parts(parts)
    b0 = sp.info()["list_builds"]
    for step in range(3):
        sp.drift(D, P)
        o, _ = _oracle_drift(o, xp, D)
        sp.reset_acceleration(P)
        nf = sp.force(P)
        gf = abi.copy_parts(parts)
        sp.download(gf, abi.FIELDS_FORCE)
        of = abi.copy_parts(o)
        of["a_hydro"] = 0
        of["u_dt"] = 0
        of["h_dt"] = 0
        of["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
        assert nf == O.fn("f64", "box_force")(of.ctypes.data, len(of), C.byref(P), None)
        # after the first step the two states drift apart at the float
        # rounding of the previous loop's h_dt (the drift reads it)
        for f in ("a_hydro", "u_dt", "h_dt"):
            assert_close(gf[f], of[f], 5e-5 if step == 0 else 2e-4, 1e-4 if step == 0 else 1e-3,
                         f"{f} step {step}")
        assert np.array_equal(gf["min_ngb_time_bin"], of["min_ngb_time_bin"])
        # the next drift reads this loop's h_dt / a_hydro on the GPU: the
        # oracle state follows its own loop's outputs the same way
        o = of
    builds = sp.info()["list_builds"] - b0
    # the density loop on the same lists (kept, or checked and rebuilt)
    sp.init_parts(P)
    nd = sp.density(P)
    gd = abi.copy_parts(parts)
    sp.download(gd, abi.FIELDS_DENSITY)
    sp.close()
    od = abi.copy_parts(o)
    O.fn("f32", "init_parts")(od.ctypes.data, len(od), C.byref(P))
    assert nd == O.fn("f64", "box_density")(od.ctypes.data, len(od), C.byref(P), None)
    for f in ("rho", "rho_dh", "wcount", "wcount_dh"):  # states apart since step 1
        assert_close(gd[f], od[f], 1e-4, 1e-4, f)
    if expect_rebuilds:
        assert builds >= 2, builds
    else:
        assert builds == 1, builds  # built at the first force loop, then kept


def test_kept_lists_follow_inactive_h_growth_vs_f64(gpu_ctx):
    """Kept lists must cover the j side of DOPAIR2's r < max(H_i, H_j) for
    inactive j too: the drift grows h of every particle (drift_part's h_dt
    term, src/drift.h), active or not. Mixed time bins (bin 2 inactive at
    max_active_bin 1), no list skin, no displacement (v_full = 0, so D = 0),
    the inactive particles' h grows by w1 = 0.1 (the active ones move by
    their own force-loop h_dt only). A check that looks at active particles
    alone keeps the lists and loses the pairs H_j,build < r < H_j,now. Both
    sides run force -> drift -> force; the second force loop must match the
    fp64 oracle's count, a_hydro, u_dt, h_dt and min_ngb_time_bin."""
    from swift_subtask_dev_amd import lib
    parts, P = _stepped_state(gpu_ctx, n=14, seed=14)
    N = len(parts)
    rng = np.random.Generator(np.random.PCG64(17))
    inactive = rng.uniform(size=N) < 0.4
    parts["time_bin"] = np.where(inactive, 2, 1).astype(np.int8)
    P.max_active_bin = 1
    dt = 1e-3
    parts["h_dt"] = np.where(inactive, 0.1 * parts["h"] / dt, 0.0).astype(np.float32)
    xp = abi.new_xparts(N)  # v_full = 0, a_grav = 0: nothing moves
    D = abi.DriftParams(dt, 0.0, 0.0, 0.0, 0.0)
    sp = lib.HydroSpace(gpu_ctx)
    sp.set_tuning(1, 0, 0, list_skin=0.0, list_keep=1)
    sp.upload(abi.copy_parts(parts))
    sp.rebuild(P)
    sp.upload_xparts(xp)
    sp.reset_acceleration(P)
    sp.force(P)  # builds the lists at the pre-drift h
    b0 = sp.info()["list_builds"]
    sp.drift(D, P)
    assert sp.info()["dx_max"] < 1e-9  # nothing moved (1e-12: the bound's floor)
    sp.reset_acceleration(P)
    nf = sp.force(P)
    gf = abi.copy_parts(parts)
    sp.download(gf, abi.FIELDS_FORCE | abi.FIELDS_DRIFT)
    builds = sp.info()["list_builds"] - b0
    sp.close()

    def reset_force(p):
        p["a_hydro"] = 0
        p["u_dt"] = 0
        p["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
        p["h_dt"] = np.where(p["time_bin"] <= P.max_active_bin, 0.0, p["h_dt"])

    o = abi.copy_parts(parts)
    reset_force(o)
    O.fn("f64", "box_force")(o.ctypes.data, N, C.byref(P), None)  # the active h_dt
    o, _ = _oracle_drift(o, xp, D)
    grown = gf["h"][inactive] / parts["h"][inactive]
    assert np.all(grown > 1.09), grown.min()
    of = abi.copy_parts(o)
    reset_force(of)
    no = O.fn("f64", "box_force")(of.ctypes.data, len(of), C.byref(P), None)
    assert nf == no
    assert builds == 1, builds  # the device check found the kept lists stale
    act = ~inactive
    for f in ("a_hydro", "u_dt", "h_dt"):
        assert_close(gf[f][act], of[f][act], 5e-5, 1e-4, f)
    assert np.array_equal(gf["min_ngb_time_bin"][act], of["min_ngb_time_bin"][act])
