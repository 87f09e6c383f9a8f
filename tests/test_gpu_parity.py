"""GPU parity: the HIP path (libswifthip, fp64) against the oracle.

Structure follows the reference's own hot-path tests:
  * test27cells (+ subset variants): runner_do{self1,pair1}_branch_density via
    the SWIFT-signature adapter vs the brute-force restatement, tolerance files
    of the reference (tests/golden/tolerance_27_*.dat);
  * test125cells: density -> ghost -> gradient -> extra ghost -> force chain,
    main cell vs the oracle chain (tolerance_125_*.dat) and vs the analytic
    solution;
  * testActivePair-style activity masks, inhibited particles, periodic wrap;
  * batch loops vs the fp64 oracle on Sedov-like boxes (tight: ~float ulp);
  * testPotentialSelf/Pair KATs through the P2P kernels; batch P2P vs oracle.

fp64 GPU vs fp32 oracle: reference tolerance files. fp64 GPU vs fp64 oracle:
relative 2e-6 (a few float ulps of the stored result; the sums differ only
in order).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import scenarios as S
from compare import compare_columns, load_tolerance, rel_err
from swift_subtask_dev_amd import abi, ics

TIGHT = 2e-6  # fp64 GPU vs fp64 oracle (stored as float)


def hydro_cols(p):
    return np.column_stack([p["rho"], p["wcount"], p["wcount_dh"], p["rho_dh"], p["div_v"],
                            p["rot_v"]])


def assert_hydro_close(g, o, rel, what="", vel_floor=1e-6, vel_rel=None):
    """Density-loop outputs; the velocity-derivative columns (div_v, rot_v)
    share one floor (vel_floor x their largest value): a divergence-free or
    curl-free field leaves pure round-off in the other, meaningless as a
    relative error."""
    assert_close(hydro_cols(g)[:, :4], hydro_cols(o)[:, :4], rel, 1e-6, what)
    vel = np.column_stack([o["div_v"], o["rot_v"]])
    floor = vel_floor * max(np.abs(vel).max(), 1e-30)
    a = np.column_stack([g["div_v"], g["rot_v"]])
    e = np.abs(a - vel) / np.maximum(np.abs(vel), floor)
    vr = rel if vel_rel is None else vel_rel
    assert e.max() <= vr, f"{what} div/rot: rel {e.max():.3e}"


def assert_close(a, b, rel, floor_frac=1e-6, what=""):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.ndim == 1:
        a, b = a[:, None], b[:, None]
    for j in range(a.shape[1]):
        fl = floor_frac * max(np.abs(b[:, j]).max(), 1e-300)
        e = rel_err(a[:, j], b[:, j], fl)
        k = int(np.argmax(e))
        assert e[k] <= rel, f"{what} col {j}: rel {e[k]:.3e} at {k}: {a[k, j]!r} vs {b[k, j]!r}"


# ---------------------------------------------------------------------------
# 125-cell chain (shared with tests/test_oracle.py for the analytic check)
# ---------------------------------------------------------------------------
def build125(vel="zero", press="const", n=6, pert=0.0, seed=0):
    rho = 2.5
    parts, bounds, locs = S.cells_grid(5, n, size=1.0, h=1.23485, rho=rho, pert=pert,
                                       vel="zero", seed=seed, shuffle=False)
    x = parts["x"]
    if vel == "const":
        parts["v"] = (1.0, 0.0, 0.0)
    elif vel == "divergent":
        parts["v"] = (x - 2.5).astype(np.float32)
    elif vel == "rotating":
        v = np.zeros_like(x)
        v[:, 0] = x[:, 1]
        v[:, 1] = -x[:, 0]
        parts["v"] = v.astype(np.float32)
    if press == "const":
        P = np.full(len(parts), 1.5)
    elif press == "gradient":
        P = 1.5 * x[:, 0]
    else:
        P = np.sqrt(((x - 2.5) ** 2).sum(axis=1)) + 1.5
    parts["u"] = (P / ((5.0 / 3.0 - 1.0) * rho)).astype(np.float32)
    parts["time_bin"] = 1
    Pp = abi.default_hydro_params((5.0, 5.0, 5.0), periodic=False, h_tolerance=1.0,
                                  max_smoothing_iterations=10)
    return parts, bounds, Pp


def run125_oracle(vel="zero", press="const", prec="f32", pert=0.0):
    parts, bounds, P = build125(vel, press, pert=pert)
    N = len(parts)
    f = lambda n: O.fn(prec, n)  # noqa: E731
    f("init_parts")(parts.ctypes.data, N, C.byref(P)) if prec == "f32" else None
    S.zero_density_fields(parts)
    nd = f("box_density")(parts.ctypes.data, N, C.byref(P), None)
    nf = C.c_longlong(0)
    f("box_ghost")(parts.ctypes.data, N, C.byref(P), C.byref(nf))
    parts["laplace_u"] = 0
    f("box_gradient")(parts.ctypes.data, N, C.byref(P), None)
    f("box_extra_ghost")(parts.ctypes.data, N, C.byref(P))
    f("box_force")(parts.ctypes.data, N, C.byref(P), None)
    f("box_end_force")(parts.ctypes.data, N, C.byref(P))
    s, e = bounds[62]
    return {"parts": parts, "main": parts[s:e].copy(), "n_density": nd}


def run125_gpu(ctx, vel="zero", press="const", pert=0.0):
    from swift_subtask_dev_amd import lib
    parts, bounds, P = build125(vel, press, pert=pert)
    S.zero_density_fields(parts)
    sp = lib.HydroSpace(ctx)
    sp.upload(parts)
    sp.rebuild(P)
    steps = sp.hydro_step(P)
    sp.download(parts, abi.FIELDS_ALL)
    sp.close()
    s, e = bounds[62]
    return {"parts": parts, "main": parts[s:e].copy(), "steps": steps}


def cols125(p):
    # test125cells.c dump columns that the SPHENIX path defines (h, rho, div_v,
    # u, P, c, a_x..a_z, h_dt, v_sig, du/dt)
    return np.column_stack([p["h"], p["rho"], p["div_v"], p["u"], p["pressure"],
                            p["soundspeed"], p["a_hydro"], p["h_dt"], p["v_sig"], p["u_dt"]])


def tol125(name):
    names, at, rt, lt = load_tolerance(name)
    pick = ["h", "rho", "div_v", "u", "P", "c", "a_x", "a_y", "a_z", "h_dt", "v_sig", "du/dt"]
    idx = [names.index(c) for c in pick]
    return pick, at[idx], rt[idx], lt[idx]


# ---------------------------------------------------------------------------
# GPU tests
# ---------------------------------------------------------------------------
CASES27_GPU = [
    ("zero", 0.0, 0.0, "tolerance_27_normal.dat"),
    ("random", 0.0, 0.0, "tolerance_27_normal.dat"),
    ("divergent", 0.0, 0.0, "tolerance_27_normal.dat"),
    ("rotating", 0.0, 0.0, "tolerance_27_normal.dat"),
    ("random", 1.1, 0.0, "tolerance_27_perturbed_h.dat"),
    ("divergent", 1.3, 0.0, "tolerance_27_perturbed_h2.dat"),
    ("rotating", 0.0, 0.1, "tolerance_27_perturbed.dat"),
]


@pytest.fixture(scope="module")
def adapter():
    from swift_subtask_dev_amd import lib
    ad = lib.load_adapter()
    assert ad.swifthip_swift_init(0, 0) == 0
    yield ad


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f32", "f64"])
@pytest.mark.parametrize("subset", [False, True])
@pytest.mark.parametrize("vel,h_pert,pert,tol", CASES27_GPU)
def test_27cells_adapter(adapter, vel, h_pert, pert, tol, subset, precision):
    """test27cells.c (and its -DTEST_DO{SELF,PAIR}_SUBSET build): the GPU
    adapter vs the brute-force float oracle with the reference's tolerance
    files, relative columns x1.5: the reference tuned them on its own srand(0)
    draws; on other draws float rounding of cancelling sums (div_v ~1e-4 for
    the random velocity field) reaches 1.1-1.6x. The fp64 path is also held to
    the fp64 oracle at 2e-6 in test_27cells_adapter_vs_f64."""
    assert adapter.swifthip_swift_set_precision(1 if precision == "f32" else 0) == 0
    P = abi.default_hydro_params((3.0, 3.0, 3.0), True)
    parts, bounds, locs = S.cells_grid(3, 6, vel=vel, h_pert=h_pert, pert=pert, seed=1)
    g = abi.copy_parts(parts)
    b = abi.copy_parts(parts)
    S.zero_density_fields(g)
    S.zero_density_fields(b)
    S.run27(g, bounds, locs, "adapter", P, subset=subset)
    S.run27(b, bounds, locs, "brute", P)
    s, e = bounds[13]
    mg, mb = abi.copy_parts(g[s:e]), abi.copy_parts(b[s:e])
    S.end_calculation(mg, P)
    S.end_calculation(mb, P)
    names, at, rt, lt = load_tolerance(tol)
    rt = rt * 1.5
    errs = compare_columns(S.density_columns(mb), S.density_columns(mg), at, rt, lt, names)
    adapter.swifthip_swift_set_precision(0)
    assert not errs, "\n".join(errs)


@pytest.mark.gpu
@pytest.mark.parametrize("vel,h_pert,pert,tol", CASES27_GPU + [("divergent", 1.2, 0.1, None)])
def test_27cells_adapter_vs_f64(adapter, vel, h_pert, pert, tol):
    """The fp64 adapter against the fp64 oracle at float-ulp tolerance (2e-6,
    div_v/rot_v floored at 1e-6 of their largest value) on every test27cells
    case, on draw 3: the draw on which the reference's own float algorithm
    misses its tolerance files by 3.6x (test_oracle.py::
    test_reference_tolerances_are_draw_specific), so the x1.5 slack of the
    float comparison above is about float rounding, not about this path."""
    P = abi.default_hydro_params((3.0, 3.0, 3.0), True)
    parts, bounds, locs = S.cells_grid(3, 6, vel=vel, h_pert=h_pert, pert=pert, seed=3)
    g = abi.copy_parts(parts)
    S.zero_density_fields(g)
    S.run27(g, bounds, locs, "adapter", P)
    # fp64 oracle on the 27-cell periodic box, main cell only
    o = abi.copy_parts(parts)
    S.zero_density_fields(o)
    s, e = bounds[13]
    O.fn("f64", "box_density_subset")(o.ctypes.data, len(o), C.byref(P),
                                      np.arange(s, e, dtype=np.int32).ctypes.data, e - s)
    # per-task mode adds each of the 27 tasks' partial sums into the float
    # fields (as SWIFT's runners do): the cancelling div/rot sums of random
    # and rotating fields keep ~27 float roundings of partials up to ~10x
    # the result (measured 1.4e-5): div/rot at 3e-5 above a floor of 1e-3 of
    # their largest value; rho, wcount and the h-derivatives stay at 2e-6
    assert_hydro_close(g[s:e], o[s:e], TIGHT, "27cells f64", vel_floor=1e-3, vel_rel=3e-5)


@pytest.mark.gpu
def test_periodic_reach_over_half_box_is_an_error(gpu_ctx):
    """A kernel reach >= half the periodic box would need more than the
    nearest image: rebuild refuses it with SWH_ERR_CELL_SMALL ("Cell smaller
    than smoothing length", runner_doiact_functions_hydro.h:2283) instead of
    silently dropping images. 4^3 lattice in a unit box: gamma*h = 0.56."""
    from swift_subtask_dev_amd import ics, lib
    parts = ics.sedov_slabs(4, 1)
    P = abi.default_hydro_params((1.0, 1.0, 1.0), True)
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(parts)
    with pytest.raises(lib.SwhError) as e:
        sp.rebuild(P)
    assert e.value.status == 4  # SWH_ERR_CELL_SMALL
    with pytest.raises(lib.SwhError):  # the loops refuse an unbuilt space
        sp.density(P)
    sp.close()
    parts = ics.sedov_slabs(6, 1)  # gamma*h = 0.376: fine
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(parts)
    sp.rebuild(P)
    sp.close()


@pytest.mark.gpu
def test_unsorted_cells_error(adapter):
    """DOPAIR1_BRANCH's "Interacting unsorted cells." precondition."""
    P = abi.default_hydro_params((3.0, 3.0, 3.0), True)
    parts, bounds, locs = S.cells_grid(3, 4, seed=3)
    eb = abi.EngineBundle(dim=(3.0, 3.0, 3.0), periodic=True, params=P)
    cs = O.CellSet(parts, bounds, locs, 1.0)  # not sorted
    adapter.swifthip_swift_clear_error()
    adapter.runner_dopair1_branch_density(C.addressof(eb.runner), cs.ptr(13), cs.ptr(14))
    assert adapter.swifthip_swift_last_error() == b"Interacting unsorted cells."
    adapter.swifthip_swift_clear_error()


@pytest.mark.gpu
@pytest.mark.parametrize("vel", ["zero", "const", "divergent", "rotating"])
@pytest.mark.parametrize("press", ["const", "gradient", "divergent"])
def test_125cells_chain(gpu_ctx, vel, press):
    """test125cells.c chain on the batch path vs the f32 oracle chain
    (tolerance_125_normal.dat) and the analytic fields."""
    gr = run125_gpu(gpu_ctx, vel, press)
    orc = run125_oracle(vel, press, "f32")
    names, at, rt, lt = tol125("tolerance_125_normal.dat")
    errs = compare_columns(cols125(orc["main"]), cols125(gr["main"]), at, rt, lt, names)
    assert not errs, "\n".join(errs)
    assert np.allclose(gr["main"]["rho"], 2.5, rtol=1e-2)  # SPH lattice estimate
    if vel == "divergent":
        assert np.allclose(gr["main"]["div_v"], 3.0, rtol=2e-2)
    if press == "gradient":
        assert np.allclose(gr["main"]["a_hydro"][:, 0], -0.6, rtol=3e-2)


@pytest.mark.gpu
def test_125cells_chain_vs_f64(gpu_ctx):
    gr = run125_gpu(gpu_ctx, "divergent", "divergent", pert=0.1)
    orc = run125_oracle("divergent", "divergent", "f64", pert=0.1)
    for f in ("h", "rho", "pressure", "soundspeed", "v_sig", "u_dt", "h_dt"):
        assert_close(gr["main"][f], orc["main"][f], 1e-5, 1e-5, f)
    assert_close(gr["main"]["a_hydro"], orc["main"]["a_hydro"], 1e-5, 1e-3, "a_hydro")


# loop_variant 7 = pair lists (the default and only loop: density builds the
# step's lists, every loop walks them); the round-1 tile loops (variants 1,
# 4, 5) were removed from the product
VARIANTS = [7]


def box_chain_gpu(ctx, parts, P, cell_factor=1, variant=0, group_size=0, **tuning):
    from swift_subtask_dev_amd import lib
    g = abi.copy_parts(parts)
    sp = lib.HydroSpace(ctx)
    sp.set_tuning(cell_factor, variant, group_size, **tuning)
    sp.upload(g)
    sp.rebuild(P)
    res = sp.hydro_step(P)
    sp.download(g, abi.FIELDS_ALL)
    sp.close()
    return g, res


def box_chain_oracle(parts, P, prec="f64"):
    o = abi.copy_parts(parts)
    N = len(o)
    f = lambda n: O.fn(prec, n)  # noqa: E731
    O.fn("f32", "init_parts")(o.ctypes.data, N, C.byref(P))
    nd = f("box_density")(o.ctypes.data, N, C.byref(P), None)
    nfail = C.c_longlong(0)
    it = f("box_ghost")(o.ctypes.data, N, C.byref(P), C.byref(nfail))
    o["laplace_u"] = 0
    ng = f("box_gradient")(o.ctypes.data, N, C.byref(P), None)
    f("box_extra_ghost")(o.ctypes.data, N, C.byref(P))
    nf = f("box_force")(o.ctypes.data, N, C.byref(P), None)
    f("box_end_force")(o.ctypes.data, N, C.byref(P))
    return o, {"density": nd, "gradient": ng, "force": nf, "ghost_iterations": it}


@pytest.mark.gpu
@pytest.mark.parametrize("variant,group_size,skin",
                         [(7, 16, 0.1), (7, 16, 0.0), (7, 16, 0.5), (0, 0, 0.0)])
@pytest.mark.parametrize("cell_factor", [1, 2, 3])
def test_box_density_vs_f64(gpu_ctx, cell_factor, variant, group_size, skin):
    """Batch density loop on a periodic Sedov-like box vs the fp64 oracle;
    identical interaction count; every grid refinement gives the same sums."""
    from swift_subtask_dev_amd import lib
    P = abi.default_hydro_params()
    parts = ics.sedov_box(20, velocity="divergent", seed=11)
    g = abi.copy_parts(parts)
    sp = lib.HydroSpace(gpu_ctx)
    sp.set_tuning(cell_factor, variant, group_size, list_skin=skin)
    sp.upload(g)
    sp.rebuild(P)
    sp.init_parts(P)
    n = sp.density(P)
    sp.download(g, abi.FIELDS_DENSITY)
    o = abi.copy_parts(parts)
    O.fn("f32", "init_parts")(o.ctypes.data, len(o), C.byref(P))
    no = O.fn("f64", "box_density")(o.ctypes.data, len(o), C.byref(P), None)
    assert n == no
    assert_hydro_close(g, o, TIGHT, "box density")


@pytest.mark.gpu
@pytest.mark.parametrize("variant,group_size,tuning",
                         [(7, 16, {}), (7, 16, {"list_skin": 0.1}), (7, 16, {"list_skin": 0.0}),
                          (7, 16, {"list_capacity": 24}), (0, 0, {"list_keep": 1})])
def test_box_chain_vs_f64(gpu_ctx, variant, group_size, tuning):
    """Full SPHENIX chain (density, ghost with h iteration, gradient, extra
    ghost, force, end force) on a perturbed box with h off-target so the
    ghost iterates."""
    P = abi.default_hydro_params()
    parts = ics.sedov_box(16, velocity="divergent", pert=0.3, seed=5)
    parts["h"] *= np.random.Generator(np.random.PCG64(1)).uniform(0.8, 1.25, len(parts))
    g, rg = box_chain_gpu(gpu_ctx, parts, P, variant=variant, group_size=group_size, **tuning)
    o, ro = box_chain_oracle(parts, P)
    assert rg["ghost_iterations"] >= 2
    # Chain tolerance: the GPU keeps struct-part (float) storage between the
    # density loop and the ghost, the fp64 oracle keeps doubles inside its
    # ghost; h agrees to ~1e-7 and the forces to ~1e-5.
    assert_close(g["h"], o["h"], 1e-6, what="h")
    for f in ("rho", "pressure", "soundspeed", "balsara", "v_sig", "laplace_u",
              "visc_alpha", "diff_alpha"):
        assert_close(g[f], o[f], 5e-5, 1e-4, f)
    # grad-h term: f is a cancelling rho_dh sum and enters the force only as
    # f_ij = 1 - f_i/m_j (~1): floor |f| at 1e-3 m, i.e. an absolute error of
    # 5e-8 in f_ij (float epsilon). The f32 oracle differs from the f64 one by
    # 1.9e-2 under the 1e-5 m floor on this case; the GPU's fp64 path by 4e-4.
    e = np.abs(g["f"] - o["f"]) / np.maximum(np.abs(o["f"]), 1e-3 * o["mass"])
    assert e.max() < 5e-5, e.max()
    assert_close(g["a_hydro"], o["a_hydro"], 5e-5, 1e-4, "a_hydro")
    assert_close(g["u_dt"], o["u_dt"], 5e-5, 1e-4, "u_dt")
    assert_close(g["h_dt"], o["h_dt"], 5e-5, 1e-4, "h_dt")
    assert np.array_equal(g["min_ngb_time_bin"], o["min_ngb_time_bin"])
    assert rg["force"] == ro["force"]


@pytest.mark.gpu
def test_box_active_mask_and_inhibited(gpu_ctx):
    """Activity (time_bin > max_active_bin: not updated, still a neighbour)
    and inhibited particles (never a neighbour), testActivePair-style."""
    from swift_subtask_dev_amd import lib
    P = abi.default_hydro_params(max_active_bin=1)
    parts = ics.sedov_box(16, velocity="random", seed=9)
    rng = np.random.Generator(np.random.PCG64(1506434777))
    parts["time_bin"] = np.where(rng.uniform(size=len(parts)) < 0.4, 2, 1)
    inh = rng.choice(len(parts), 40, replace=False)
    parts["time_bin"][inh] = abi.TIME_BIN_INHIBITED
    parts["rho"] = 7.0  # inactive particles must keep this
    g = abi.copy_parts(parts)
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(g)
    sp.rebuild(P)
    sp.init_parts(P)
    n = sp.density(P)
    sp.download(g, abi.FIELDS_DENSITY)
    o = abi.copy_parts(parts)
    O.fn("f32", "init_parts")(o.ctypes.data, len(o), C.byref(P))
    no = O.fn("f64", "box_density")(o.ctypes.data, len(o), C.byref(P), None)
    assert n == no
    inactive = g["time_bin"] != 1
    assert np.all(g["rho"][inactive] == 7.0)
    act = ~inactive
    assert_hydro_close(g[act], o[act], TIGHT, "active")


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_non_periodic_box(gpu_ctx, variant):
    P = abi.default_hydro_params(periodic=False)
    parts = ics.sedov_box(14, velocity="divergent", seed=21)
    g, rg = box_chain_gpu(gpu_ctx, parts, P, variant=variant)
    o, ro = box_chain_oracle(parts, P)
    assert rg["density"] == ro["density"]
    assert_close(g["rho"], o["rho"], 1e-5, what="rho")
    assert_close(g["a_hydro"], o["a_hydro"], 5e-5, 1e-4, "a_hydro")


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_clustered_box_chain(gpu_ctx, variant):
    """EAGLE-like stand-in: smoothing lengths spanning >10x after the ghost
    (dense clumps overflow the two-phase hit lists mid-row)."""
    P = abi.default_hydro_params()
    parts = ics.clustered_box(12, n_clumps=3, per_clump=600, seed=4)
    g, rg = box_chain_gpu(gpu_ctx, parts, P, variant=variant)
    o, ro = box_chain_oracle(parts, P)
    assert g["h"].max() / g["h"].min() > 5
    assert_close(g["h"], o["h"], 1e-5, what="h")
    assert_close(g["rho"], o["rho"], 1e-4, what="rho")
    assert_close(g["a_hydro"], o["a_hydro"], 1e-4, 1e-3, "a_hydro")


@pytest.fixture(scope="module")
def clustered_state(gpu_ctx):
    """A clustered box (24^3 background + 6 clumps of 6,000) with h converged
    by the GPU chain: H_max / H_typical > 1.5, so the grid is sized by the
    typical H and the list build prunes cells by their own H_max."""
    P = abi.default_hydro_params()
    parts = ics.clustered_box(24, n_clumps=6, per_clump=6000, seed=9)
    g, res = box_chain_gpu(gpu_ctx, parts, P)
    return g, P


@pytest.mark.gpu
@pytest.mark.parametrize("capacity", [0, 24])
def test_clustered_adaptive_grid_loops_vs_f64(gpu_ctx, clustered_state, capacity):
    """Density and force on the clustered box vs the fp64 oracle, every
    particle, exact interaction counts; capacity 24 sends hundreds of
    particles through the wave-per-particle overflow search."""
    from swift_subtask_dev_amd import lib
    parts, P = clustered_state
    g = abi.copy_parts(parts)
    sp = lib.HydroSpace(gpu_ctx)
    sp.set_tuning(list_capacity=capacity)
    sp.upload(g)
    sp.rebuild(P)
    info = sp.info()
    assert g["h"].max() / g["h"].min() > 10
    sp.init_parts(P)
    nd = sp.density(P)
    if capacity:
        assert sp.info()["list_overflow"] > 100
    sp.download(g, abi.FIELDS_DENSITY)
    sp.close()
    o = abi.copy_parts(parts)
    O.fn("f32", "init_parts")(o.ctypes.data, len(o), C.byref(P))
    assert nd == O.fn("f64", "box_density")(o.ctypes.data, len(o), C.byref(P), None)
    assert_hydro_close(_by_id(g), _by_id(o), TIGHT, "clustered density")
    # force on the converged chain state (its force-side union fields intact)
    gf = abi.copy_parts(parts)
    sp = lib.HydroSpace(gpu_ctx)
    sp.set_tuning(list_capacity=capacity)
    sp.upload(gf)
    sp.rebuild(P)
    sp.reset_acceleration(P)
    nf = sp.force(P)
    sp.download(gf, abi.FIELDS_FORCE)
    sp.close()
    of = abi.copy_parts(parts)
    of["a_hydro"] = 0
    of["u_dt"] = 0
    of["h_dt"] = 0
    of["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
    assert nf == O.fn("f64", "box_force")(of.ctypes.data, len(of), C.byref(P), None)
    a, b = _by_id(gf), _by_id(of)
    assert_close(a["a_hydro"], b["a_hydro"], 5e-5, 1e-4, "a_hydro")
    assert_close(a["u_dt"], b["u_dt"], 5e-5, 1e-4, "u_dt")
    assert np.array_equal(a["min_ngb_time_bin"], b["min_ngb_time_bin"])
    assert info["cdim"][0] > 1.0 / (float(parts["h"].max()) * 1.825742) * 1.3


@pytest.mark.gpu
@pytest.mark.parametrize("bins", ["mixed", "one_low"])
def test_force_min_ngb_time_bin(gpu_ctx, clustered_state, bins):
    """The time-bin limiter of the force loop (runner_iact_nonsym_timebin):
    mixed bins 3/4/6 with random initial minima (some under every bin
    present), and one particle alone in bin 2 among bin-5 particles:
    min_ngb_time_bin equal to the f64 oracle's, exact counts."""
    from swift_subtask_dev_amd import lib
    parts, _ = clustered_state
    P = abi.default_hydro_params(max_active_bin=abi.NUM_TIME_BINS)
    rng = np.random.Generator(np.random.PCG64(2024 + len(bins)))
    n = len(parts)
    base = abi.copy_parts(parts)
    base["time_bin"] = rng.choice([3, 4, 6], n) if bins == "mixed" else 5
    if bins == "one_low":
        base["time_bin"][n // 2] = 2
    base["time_bin"][rng.choice(n, 30, replace=False)] = abi.TIME_BIN_INHIBITED
    # the initial minima stay (no reset_acceleration: the force adds into
    # the zeroed accumulators of the upload)
    base["min_ngb_time_bin"] = rng.choice([2, 3, 5, abi.NUM_TIME_BINS + 1], n)
    base["a_hydro"] = 0
    base["u_dt"] = 0
    base["h_dt"] = 0
    gf = abi.copy_parts(base)
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(gf)
    sp.rebuild(P)
    nf = sp.force(P)
    sp.download(gf, abi.FIELDS_FORCE)
    sp.close()
    of = abi.copy_parts(base)
    assert nf == O.fn("f64", "box_force")(of.ctypes.data, len(of), C.byref(P), None)
    a, b = _by_id(gf), _by_id(of)
    live = a["time_bin"] != abi.TIME_BIN_INHIBITED
    assert np.array_equal(a["min_ngb_time_bin"][live], b["min_ngb_time_bin"][live])
    assert_close(a["a_hydro"][live], b["a_hydro"][live], 5e-5, 1e-4, "a_hydro")
    if bins == "one_low":  # the bin-2 particle's neighbours took its bin
        assert (b["min_ngb_time_bin"][live] == 2).sum() > 10


# ---------------------------------------------------------------------------
# Per-task force / gradient through the adapter on prepared inputs
# ---------------------------------------------------------------------------
def prepared_27cells(seed=4, vel="divergent", h_pert=1.2, pert=0.1):
    """27 cells whose force-side fields (rho, P, c, f, balsara, alphas) are
    set to physical random values, as after the extra ghost."""
    parts, bounds, locs = S.cells_grid(3, 5, vel=vel, h_pert=h_pert, pert=pert, seed=seed)
    rng = np.random.Generator(np.random.PCG64(seed))
    n = len(parts)
    parts["rho"] = rng.uniform(0.8, 1.2, n)
    parts["u"] = rng.uniform(0.5, 1.5, n)
    parts["pressure"] = (2.0 / 3.0) * parts["u"] * parts["rho"]
    parts["soundspeed"] = np.sqrt(5.0 / 3.0 * parts["pressure"] / parts["rho"])
    parts["f"] = rng.uniform(-0.05, 0.05, n) * parts["mass"]
    parts["balsara"] = rng.uniform(0, 1, n)
    parts["visc_alpha"] = rng.uniform(0, 1, n)
    parts["diff_alpha"] = rng.uniform(0, 0.5, n)
    parts["a_hydro"] = 0
    parts["u_dt"] = 0
    parts["h_dt"] = 0
    parts["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
    return parts, bounds, locs


@pytest.mark.gpu
def test_force_pair_self_adapter(adapter):
    """DOPAIR2/DOSELF2 (+ time-bin limiter) of the main cell against its 26
    neighbours: GPU adapter vs the oracle's sorted DOPAIR2/DOSELF2 (f32,
    tolerance_125 a/u_dt/h_dt columns) and the brute-force pairs_all_force."""
    P = abi.default_hydro_params((3.0, 3.0, 3.0), True)
    parts, bounds, locs = prepared_27cells()
    rng = np.random.Generator(np.random.PCG64(77))
    parts["time_bin"] = np.where(rng.uniform(size=len(parts)) < 0.3, 2, 1)
    P.max_active_bin = 2  # all active; time bins differ -> limiter min is 1
    g = abi.copy_parts(parts)
    b = abi.copy_parts(parts)
    eb = abi.EngineBundle(dim=(3.0, 3.0, 3.0), periodic=True, params=P, max_active_bin=2)
    cg = O.CellSet(g, bounds, locs, 1.0)
    cg.sort_all()
    adapter.swifthip_swift_clear_error()
    for j in range(27):
        if j != 13:
            adapter.runner_dopair2_branch_force(C.addressof(eb.runner), cg.ptr(13), cg.ptr(j))
    adapter.runner_doself2_branch_force(C.addressof(eb.runner), cg.ptr(13))
    assert not adapter.swifthip_swift_last_error()
    cb = O.CellSet(b, bounds, locs, 1.0)
    for j in range(27):
        if j != 13:
            O.fn("f32", "pairs_all_force")(C.addressof(eb.runner), cb.ptr(13), cb.ptr(j))
    O.fn("f32", "self_all_force")(C.addressof(eb.runner), cb.ptr(13))
    s, e = bounds[13]
    cols = lambda p: np.column_stack([p["a_hydro"], p["u_dt"], p["h_dt"]])  # noqa: E731
    names = ["a_x", "a_y", "a_z", "du/dt", "h_dt"]
    # tolerance_125 rel 1e-4, x3: these random (non-smooth) force inputs make
    # the float oracle's sums cancel harder than test125cells' smooth fields
    at = np.full(5, 1e-4)
    rt = np.full(5, 3e-4)
    lt = np.full(5, 1e-4)
    errs = compare_columns(cols(b[s:e]), cols(g[s:e]), at, rt, lt, names)
    assert not errs, "\n".join(errs)
    assert np.array_equal(g["min_ngb_time_bin"][s:e], b["min_ngb_time_bin"][s:e])
    cg.free_sorts()
    # fp64 GPU vs fp64 oracle (all 27 cells' force loop, main cell compared).
    # Per-task mode writes each task's fp64 partial sum back into struct
    # part's float fields (26 pair tasks + 1 self task, as SWIFT's runners
    # do), so a cancelling sum carries ~27 float roundings of partial sums
    # up to ~100x the final value: rel 1e-4 (observed 5.5e-5), not TIGHT.
    # The batch loops, which sum in fp64 across all tasks, are held to TIGHT.
    o = abi.copy_parts(parts)
    O.fn("f64", "box_force")(o.ctypes.data, len(o), C.byref(P), None)
    assert_close(cols(g[s:e]), cols(o[s:e]), 1e-4, 1e-6, "force f64 (per-task)")
    assert np.array_equal(g["min_ngb_time_bin"][s:e], o["min_ngb_time_bin"][s:e])


# ---------------------------------------------------------------------------
# Gravity
# ---------------------------------------------------------------------------
@pytest.mark.gpu
def test_potential_self_kat_gpu(adapter):
    from test_oracle import _acceleration, _check_kat, _potential, potential_self_gparts
    g = potential_self_gparts()
    cell = abi.Cell()
    cell.width[:] = (1.0, 1.0, 1.0)
    cell.grav.parts = g.ctypes.data
    cell.grav.count = len(g)
    mp = abi.GravityTensors(CoM=(C.c_double * 3)(0, 0.5, 0.5), r_max=0.0)
    cell.grav.multipole = C.pointer(mp)
    cell.grav.ti_end_min = 8
    eb = abi.EngineBundle(dim=(10.0, 10.0, 10.0), periodic=False)
    adapter.runner_doself_grav_pp(C.addressof(eb.runner), C.addressof(cell))
    assert not adapter.swifthip_swift_last_error()
    big = np.finfo(np.float32).max
    for n in range(1, 101):
        x = g["x"][n, 0]
        assert _check_kat(g["potential"][n], _potential(1.0, x, 0.02, big), 1e-6, 1e-6)
        assert _check_kat(g["a_grav"][n, 0], _acceleration(1.0, x, 0.02, big), 1e-6, 1e-6)


@pytest.mark.gpu
def test_potential_pair_kat_gpu(adapter):
    from test_oracle import _acceleration, _check_kat, _potential, potential_pair_gparts
    gi, gj = potential_pair_gparts()
    cells = (abi.Cell * 2)()
    mps = [abi.GravityTensors(CoM=(C.c_double * 3)(0, 0.5, 0.5), r_max=0.1),
           abi.GravityTensors(CoM=(C.c_double * 3)(1.5, 0.5, 0.5), r_max=0.1)]
    for c, g, mp, loc in ((cells[0], gi, mps[0], 0.0), (cells[1], gj, mps[1], 1.0)):
        c.loc[0] = loc
        c.width[:] = (1.0, 1.0, 1.0)
        c.grav.parts = g.ctypes.data
        c.grav.count = len(g)
        c.grav.multipole = C.pointer(mp)
        c.grav.ti_end_min = 8
    eb = abi.EngineBundle(dim=(10.0, 10.0, 10.0), periodic=False)
    adapter.runner_dopair_grav_pp(C.addressof(eb.runner), C.addressof(cells[0]),
                                  C.addressof(cells[1]), 1, 1)
    assert not adapter.swifthip_swift_last_error()
    big = np.finfo(np.float32).max
    for n in range(100):
        r = gj["x"][n, 0]
        assert _check_kat(gj["potential"][n], _potential(1.0, r, 0.1, big), 2e-6, 1e-6)
        assert _check_kat(gj["a_grav"][n, 0], _acceleration(1.0, r, 0.1, big), 2e-6, 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("periodic,truncated", [(False, 0), (True, 0), (True, 1)])
def test_grav_batch_vs_oracle(gpu_ctx, periodic, truncated):
    """Batch P2P over every leaf and its 26 neighbours vs the oracle's
    runner_doself_grav_pp / runner_dopair_grav_pp (fp64 build)."""
    from swift_subtask_dev_amd import lib
    gp = ics.uniform_gravity_box(12, epsilon=0.02, seed=3)
    cdim = 4
    gs, leaves = ics.leaf_cells(gp, cdim)
    offs, pairs = ics.neighbour_pairs(cdim, periodic=periodic, truncated=truncated)
    G = abi.GravParams(1 if periodic else 0, (C.c_float * 3)(1, 1, 1),
                       1.0 / 0.3 if truncated else 0.0, 0.0 if truncated else 1e30,
                       abi.NUM_TIME_BINS)
    g = abi.copy_parts(gs)
    sp = lib.GravSpace(gpu_ctx)
    sp.upload(g)
    sp.set_leaves(leaves, offs, pairs)
    n = sp.pp(G)
    sp.download(g)
    o = abi.copy_parts(gs)
    no = O.fn("f64", "grav_pp_leaves")(o.ctypes.data, leaves.ctypes.data, len(leaves),
                                       offs.ctypes.data, pairs.ctypes.data, C.byref(G), None, None)
    assert n == no
    # net accelerations cancel strongly in a uniform box: floor at 1e-6 of the
    # largest component
    assert_close(g["a_grav"], o["a_grav"], 1e-6, 1e-6, "a_grav")
    assert_close(g["potential"], o["potential"], 1e-6, 1e-6, "potential")


# ---------------------------------------------------------------------------
# The headline configuration itself (bench.py's 128^3 input, default tuning)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def headline_state(gpu_ctx):
    """bench.py's exact input: ics.sedov_slabs(128, 1) taken through the full
    SPHENIX chain on the GPU (density, ghost, gradient, extra ghost, force),
    i.e. the converged state the bench's timed step starts from."""
    from swift_subtask_dev_amd import lib
    parts = ics.sedov_slabs(128, 1)
    P = abi.default_hydro_params((1.0, 1.0, 1.0), True)
    P.max_active_bin = 1
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(parts)
    sp.rebuild(P)
    sp.hydro_step(P)
    sp.download(parts, abi.FIELDS_ALL)
    sp.close()
    return parts, P


def _by_id(p):
    return p[np.argsort(p["id"], kind="stable")]


@pytest.mark.gpu
def test_headline_128_density_vs_f64(gpu_ctx, headline_state):
    """The bench's timed density loop (hydro_init_part + density) at 128^3 on
    the bench's own input vs the fp64 oracle, every particle: rho, wcount,
    wcount_dh, rho_dh, div_v, rot_v to 2e-6 and the exact interaction count
    (98,518,377 directed density interactions)."""
    from swift_subtask_dev_amd import lib
    parts, P = headline_state
    g = abi.copy_parts(parts)
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(g)
    sp.rebuild(P)
    sp.init_parts(P)
    n = sp.density(P)
    sp.download(g, abi.FIELDS_DENSITY)
    sp.close()
    o = abi.copy_parts(parts)
    O.fn("f32", "init_parts")(o.ctypes.data, len(o), C.byref(P))
    no = O.fn("f64", "box_density")(o.ctypes.data, len(o), C.byref(P), None)
    assert n == no == 98518377
    assert_hydro_close(_by_id(g), _by_id(o), TIGHT, "128^3 density")


@pytest.mark.gpu
def test_headline_128_force_vs_f64(gpu_ctx, headline_state):
    """The bench's timed force loop (hydro_reset_acceleration + force) at
    128^3 on the converged inputs vs the fp64 oracle: a_hydro, u_dt, h_dt to
    5e-5 (floor 1e-4 of the column maximum), min_ngb_time_bin exact, and the
    exact count (101,420,958 directed force interactions)."""
    from swift_subtask_dev_amd import lib
    parts, P = headline_state
    g = abi.copy_parts(parts)
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(g)
    sp.rebuild(P)
    sp.reset_acceleration(P)
    n = sp.force(P)
    sp.download(g, abi.FIELDS_FORCE)
    sp.close()
    o = abi.copy_parts(parts)
    o["a_hydro"] = 0
    o["u_dt"] = 0
    o["h_dt"] = 0
    o["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
    no = O.fn("f64", "box_force")(o.ctypes.data, len(o), C.byref(P), None)
    assert n == no == 101420958
    g, o = _by_id(g), _by_id(o)
    assert_close(g["a_hydro"], o["a_hydro"], 5e-5, 1e-4, "a_hydro")
    assert_close(g["u_dt"], o["u_dt"], 5e-5, 1e-4, "u_dt")
    assert_close(g["h_dt"], o["h_dt"], 5e-5, 1e-4, "h_dt")
    assert np.array_equal(g["min_ngb_time_bin"], o["min_ngb_time_bin"])


@pytest.mark.gpu
@pytest.mark.parametrize("n,cdim,periodic,truncated", [(32, 4, False, 0), (40, 5, True, 1)])
def test_grav_bench_geometry_vs_oracle(gpu_ctx, n, cdim, periodic, truncated):
    """P2P at the bench's geometry scaled down (BASELINE config 4: uniform DM
    box, softening 0.001, leaves of ~400-500 gparts, every leaf with itself and
    its 26 neighbours) vs the fp64 oracle's runner_doself/dopair_grav_pp:
    a_grav and potential to 1e-6 (floor 1e-6 of the column maximum), exact
    interaction count."""
    from swift_subtask_dev_amd import lib
    gp = ics.uniform_gravity_box(n, epsilon=0.001, seed=7)
    gs, leaves = ics.leaf_cells(gp, cdim)
    offs, pairs = ics.neighbour_pairs(cdim, periodic=periodic, truncated=truncated)
    G = abi.GravParams(1 if periodic else 0, (C.c_float * 3)(1, 1, 1),
                       1.0 / 0.3 if truncated else 0.0, 0.0 if truncated else 1e30,
                       abi.NUM_TIME_BINS)
    g = abi.copy_parts(gs)
    sp = lib.GravSpace(gpu_ctx)
    sp.upload(g)
    sp.set_leaves(leaves, offs, pairs)
    ng = sp.pp(G)
    sp.download(g)
    sp.close()
    o = abi.copy_parts(gs)
    no = O.fn("f64", "grav_pp_leaves")(o.ctypes.data, leaves.ctypes.data, len(leaves),
                                       offs.ctypes.data, pairs.ctypes.data, C.byref(G), None, None)
    assert ng == no
    assert_close(g["a_grav"], o["a_grav"], 1e-6, 1e-6, "a_grav")
    assert_close(g["potential"], o["potential"], 1e-6, 1e-6, "potential")


@pytest.mark.gpu
def test_density_list_reuse(gpu_ctx):
    """diag_mode 7: a density loop keeps still-valid pair lists; its sums equal
    a fresh build's bitwise and the oracle's count, and a rebuild (positions
    may have moved) makes the next density build again."""
    from swift_subtask_dev_amd import lib
    P = abi.default_hydro_params()
    parts = ics.sedov_box(14, velocity="divergent", seed=12)
    sp = lib.HydroSpace(gpu_ctx)
    sp.set_tuning(1, 7, 16, diag_mode=7)
    sp.upload(abi.copy_parts(parts))
    sp.rebuild(P)
    res = []
    for _ in range(2):
        g = abi.copy_parts(parts)
        sp.init_parts(P)
        n = sp.density(P)
        sp.download(g, abi.FIELDS_DENSITY)
        res.append((n, g))
    assert res[0][0] == res[1][0]
    for f in ("rho", "rho_dh", "wcount", "wcount_dh", "div_v", "rot_v"):
        assert np.array_equal(res[0][1][f], res[1][1][f]), f
    o = abi.copy_parts(parts)
    O.fn("f32", "init_parts")(o.ctypes.data, len(o), C.byref(P))
    no = O.fn("f64", "box_density")(o.ctypes.data, len(o), C.byref(P), None)
    assert res[1][0] == no
    assert_hydro_close(res[1][1], o, TIGHT, "density on reused lists")
    sp.rebuild(P)
    assert not sp.info()["list_valid"]
    sp.init_parts(P)
    assert sp.density(P) == no
    sp.close()


@pytest.mark.gpu
@pytest.mark.parametrize("adaptive", [False, True])
def test_chain_few_grown_searched(gpu_ctx, request, adaptive):
    """Converged smoothing lengths with a few cut by 30%: the ghost grows those
    back past their list reach (skin 1%), too few to rebuild every list, so
    the gradient loop searches them and the force loop also their neighbours
    within the grown H (grown_mark_kernel): one list build in the chain, and
    the chain still equals the oracle's. The clustered box runs the adaptive
    grid, whose per-cell reach the grown H must raise."""
    from swift_subtask_dev_amd import lib
    P = abi.default_hydro_params()
    if adaptive:
        parts, _ = request.getfixturevalue("clustered_state")  # h converged by the GPU
        parts = abi.copy_parts(parts)
    else:
        parts = ics.sedov_box(16, velocity="divergent", pert=0.3, seed=5)
        conv, _ = box_chain_oracle(parts, P)
        parts = abi.copy_parts(parts)
        parts["h"] = conv["h"]
    cut = np.random.Generator(np.random.PCG64(4)).choice(len(parts), 6, replace=False)
    parts["h"][cut] *= 0.7
    g = abi.copy_parts(parts)
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(g)
    sp.rebuild(P)
    b0 = sp.info()["list_builds"]
    rg = sp.hydro_step(P)
    builds = sp.info()["list_builds"] - b0
    sp.download(g, abi.FIELDS_ALL)
    sp.close()
    o, ro = box_chain_oracle(parts, P)
    assert builds == 1, builds  # the density loop's; none for the grown few
    assert rg["gradient"] == ro["gradient"] and rg["force"] == ro["force"]
    tol_h, tol = (1e-5, 1e-4) if adaptive else (1e-6, 5e-5)
    assert_close(g["h"], o["h"], tol_h, what="h")
    assert_close(g["rho"], o["rho"], tol, 1e-4, "rho")
    assert_close(g["a_hydro"], o["a_hydro"], tol, 1e-3 if adaptive else 1e-4, "a_hydro")
    assert_close(g["u_dt"], o["u_dt"], tol, 1e-3 if adaptive else 1e-4, "u_dt")
    assert np.array_equal(g["min_ngb_time_bin"], o["min_ngb_time_bin"])


@pytest.mark.gpu
def test_grown_after_larger_upload(gpu_ctx):
    """The grown-particle marks are sized to the space's particle count: a
    space that took the grown-search path at 16^3 and is then given a larger
    particle set (20^3) takes it again, with marks for every particle (the
    buffer is re-reserved and zeroed when n grows), and the chain still equals
    the oracle's."""
    from swift_subtask_dev_amd import lib
    P = abi.default_hydro_params()

    def cut_state(n, seed):
        parts = ics.sedov_box(n, velocity="divergent", pert=0.3, seed=seed)
        conv, _ = box_chain_oracle(parts, P)
        parts = abi.copy_parts(parts)
        parts["h"] = conv["h"]
        cut = np.random.Generator(np.random.PCG64(seed)).choice(len(parts), 6, replace=False)
        parts["h"][cut] *= 0.7
        return parts

    sp = lib.HydroSpace(gpu_ctx)
    for n, seed in ((16, 5), (20, 6)):
        parts = cut_state(n, seed)
        g = abi.copy_parts(parts)
        sp.upload(g)
        sp.rebuild(P)
        b0 = sp.info()["list_builds"]
        rg = sp.hydro_step(P)
        builds = sp.info()["list_builds"] - b0
        sp.download(g, abi.FIELDS_ALL)
        o, ro = box_chain_oracle(parts, P)
        assert builds == 1, (n, builds)  # the grown few searched, not rebuilt
        assert rg["gradient"] == ro["gradient"] and rg["force"] == ro["force"], n
        assert_close(g["h"], o["h"], 1e-6, what="h")
        assert_close(g["a_hydro"], o["a_hydro"], 5e-5, 1e-4, "a_hydro")
        assert np.array_equal(g["min_ngb_time_bin"], o["min_ngb_time_bin"])
    sp.close()
