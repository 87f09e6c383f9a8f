"""The Wendland C2 SPH kernel (src/kernel_hydro.h:121-147; SWIFT's
configure --with-kernel=wendland-C2, configure.ac:2107-2137, as
examples/SmallCosmoVolume/SmallCosmoVolume_lightcone/README uses it).

The kernel is a build-time choice on both sides, as in SWIFT:
libswifthip_wc2.so / libswifthip_swift_wc2.so (-DSWH_KERNEL_WENDLAND_C2) on
the GPU, liboracle_wc2_{f32,f64}.so (-DORACLE_WENDLAND_C2) in the oracle,
whose kernel is pinned to the reference's own kernel definition
(theory/SPH/Kernels/kernel_definitions.tex:143-151, kernels.py:155,222) in
tests/test_oracle.py. The tests repeat the cubic-spline parity cases with it:
test27cells through the wc2 adapter (reference tolerance files), the batch
chain (density, ghost, gradient, extra ghost, force, end force) and the 64^3
density + force loops against the fp64 wc2 oracle, exact counts.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import scenarios as S
from compare import compare_columns, load_tolerance
from test_gpu_parity import TIGHT, _by_id, assert_close, assert_hydro_close
from test_gpu_physics import check_chain, evolving_box, gpu_chain, oracle_chain
from swift_subtask_dev_amd import abi, ics

pytestmark = pytest.mark.gpu
WC2 = "wendland-c2"


@pytest.fixture(scope="module")
def ctx_wc2():
    from swift_subtask_dev_amd import lib
    ctx = lib.Context(0, "f64", kernel=WC2)
    yield ctx
    ctx.close()


@pytest.fixture(scope="module")
def adapter_wc2():
    from swift_subtask_dev_amd import lib
    ad = lib.load_adapter(WC2)
    assert ad.swifthip_swift_init(0, 0) == 0
    yield ad


def test_library_reports_its_kernel(ctx_wc2, adapter_wc2):
    """Each kernel's library and adapter stay bound to each other with both
    loaded in one process (the adapters call swh_* by name)."""
    from swift_subtask_dev_amd import lib
    assert ctx_wc2._lib.swh_kernel_name() == b"wendland-c2"
    assert lib.load().swh_kernel_name() == b"cubic-spline"
    for ad, want in ((lib.load_adapter(), b"cubic-spline"), (adapter_wc2, b"wendland-c2")):
        ad.swh_kernel_name.restype = C.c_char_p  # found in the adapter's own dependency
        assert ad.swh_kernel_name() == want


@pytest.mark.parametrize("vel,h_pert,pert,tol", [
    ("zero", 0.0, 0.0, "tolerance_27_normal.dat"),
    ("divergent", 1.1, 0.1, "tolerance_27_perturbed_h.dat"),
    ("rotating", 0.0, 0.1, "tolerance_27_perturbed.dat"),
])
def test_27cells_adapter_wc2(adapter_wc2, vel, h_pert, pert, tol):
    """test27cells with the Wendland C2 kernel: the wc2 adapter's
    runner_dopair1/doself1_branch_density in float vs the wc2 brute-force
    float oracle under the reference's tolerance files (relative x1.5, as the
    cubic case), and in fp64 vs the fp64 wc2 oracle at 2e-6. (The fp64 path
    is not held to the float files: the reference's float Horner evaluation
    of the degree-5 polynomial cancels near the edge of the support, and
    wcount_dh then differs from the exact value by ~7e-5.)"""
    P = abi.default_hydro_params((3.0, 3.0, 3.0), True)
    parts, bounds, locs = S.cells_grid(3, 6, vel=vel, h_pert=h_pert, pert=pert, seed=1)
    s, e = bounds[13]
    assert adapter_wc2.swifthip_swift_set_precision(1) == 0
    g = abi.copy_parts(parts)
    b = abi.copy_parts(parts)
    S.zero_density_fields(g)
    S.zero_density_fields(b)
    S.run27(g, bounds, locs, "adapter", P, kernel=WC2)
    S.run27(b, bounds, locs, "brute", P, kernel=WC2)
    adapter_wc2.swifthip_swift_set_precision(0)
    mg, mb = abi.copy_parts(g[s:e]), abi.copy_parts(b[s:e])
    S.end_calculation(mg, P, WC2)
    S.end_calculation(mb, P, WC2)
    names, at, rt, lt = load_tolerance(tol)
    errs = compare_columns(S.density_columns(mb), S.density_columns(mg), at, rt * 1.5, lt, names)
    assert not errs, "\n".join(errs)
    # fp64 adapter vs the fp64 wc2 oracle (raw sums of the main cell)
    g = abi.copy_parts(parts)
    S.zero_density_fields(g)
    S.run27(g, bounds, locs, "adapter", P, kernel=WC2)
    o = abi.copy_parts(parts)
    S.zero_density_fields(o)
    O.fn("f64", "box_density_subset", WC2)(o.ctypes.data, len(o), C.byref(P),
                                           np.arange(s, e, dtype=np.int32).ctypes.data, e - s)
    # per-task sums: 27 float partials per field, as SWIFT's runners add them
    # (the bars of test_gpu_parity.py::test_27cells_adapter_vs_f64)
    assert_hydro_close(g[s:e], o[s:e], TIGHT, "wc2 27cells fp64", vel_floor=1e-3, vel_rel=3e-5)
    # the kernel really is Wendland C2: the cubic oracle gives another rho
    c = abi.copy_parts(parts)
    S.zero_density_fields(c)
    S.run27(c, bounds, locs, "brute", P)
    assert np.abs(c["rho"][s:e] / b["rho"][s:e] - 1.0).max() > 1e-3


def test_box_chain_wc2_vs_f64(ctx_wc2):
    """The whole SPHENIX chain with the Wendland C2 kernel on a periodic box
    in a converging, shearing flow with mixed time bins (time_base > 0):
    exact counts, h to 1e-6, every chain field at the chain tolerances."""
    parts = evolving_box(n=16, seed=51)
    P = abi.default_hydro_params(time_base=2e-3, max_active_bin=3)
    g, rg = gpu_chain(ctx_wc2, parts, P)
    o, ro = oracle_chain(parts, P, kernel=WC2)
    check_chain(g, rg, o, ro, parts["time_bin"] <= 3)
    oc, _ = oracle_chain(parts, P)  # cubic: another h (gamma and W differ)
    assert np.abs(oc["h"] / o["h"] - 1.0).max() > 2e-3


def test_sedov64_density_force_wc2_vs_f64(ctx_wc2):
    """64^3 Sedov-like box, h converged by the wc2 chain, then the bench's
    two timed loops (density, force) vs the fp64 wc2 oracle: every particle,
    density fields to 2e-6, a_hydro / u_dt / h_dt to 5e-5, exact counts."""
    from swift_subtask_dev_amd import lib
    parts = ics.sedov_slabs(64, 1)
    P = abi.default_hydro_params((1.0, 1.0, 1.0), True)
    P.max_active_bin = 1
    sp = lib.HydroSpace(ctx_wc2)
    sp.upload(parts)
    sp.rebuild(P)
    sp.hydro_step(P)
    sp.download(parts, abi.FIELDS_ALL)
    g = abi.copy_parts(parts)
    sp.upload(g)
    sp.rebuild(P)
    sp.init_parts(P)
    nd = sp.density(P)
    sp.download(g, abi.FIELDS_DENSITY)
    gf = abi.copy_parts(parts)
    sp.upload(gf)
    sp.rebuild(P)
    sp.reset_acceleration(P)
    nf = sp.force(P)
    sp.download(gf, abi.FIELDS_FORCE)
    sp.close()
    o = abi.copy_parts(parts)
    O.fn("f32", "init_parts", WC2)(o.ctypes.data, len(o), C.byref(P))
    assert nd == O.fn("f64", "box_density", WC2)(o.ctypes.data, len(o), C.byref(P), None)
    assert_hydro_close(_by_id(g), _by_id(o), TIGHT, "wc2 64^3 density")
    of = abi.copy_parts(parts)
    of["a_hydro"] = 0
    of["u_dt"] = 0
    of["h_dt"] = 0
    of["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
    assert nf == O.fn("f64", "box_force", WC2)(of.ctypes.data, len(of), C.byref(P), None)
    gf, of = _by_id(gf), _by_id(of)
    for f in ("a_hydro", "u_dt", "h_dt"):
        assert_close(gf[f], of[f], 5e-5, 1e-4, f)
    assert np.array_equal(gf["min_ngb_time_bin"], of["min_ngb_time_bin"])
    # ~ (gamma_wc2 / gamma_cubic)^3 x the cubic spline's 47.8 directed pairs
    assert 50 < nd / len(parts) < 65, nd / len(parts)
