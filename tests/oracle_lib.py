"""Test-infrastructure bindings of the CPU oracle (oracle/oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

from swift_subtask_dev_amd import abi

REPO = Path(__file__).resolve().parents[1]
ORACLE_DIR = REPO / "oracle"
F32 = ORACLE_DIR / "_build" / "liboracle_f32.so"
F64 = ORACLE_DIR / "_build" / "liboracle_f64.so"
# the Wendland C2 SPH kernel builds (oracle/Makefile, -DORACLE_WENDLAND_C2)
WC2 = {"f32": ORACLE_DIR / "_build" / "liboracle_wc2_f32.so",
       "f64": ORACLE_DIR / "_build" / "liboracle_wc2_f64.so"}

_libs = {}


def build() -> None:
    r = subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + r.stdout + r.stderr)


class OracleParams(abi.HydroParams):
    """oracle_params has the same layout as swh_hydro_params."""


class OracleGravParams(abi.GravParams):
    pass


def load(prec: str = "f32", kernel: str = "cubic-spline") -> C.CDLL:
    key = (prec, kernel)
    if key in _libs:
        return _libs[key]
    if kernel == "cubic-spline":
        path = F32 if prec == "f32" else F64
    elif kernel == "wendland-c2":
        path = WC2[prec]
    else:
        raise ValueError(kernel)
    if not _libs:
        build()  # incremental make: picks up oracle.c edits
    lib = C.CDLL(str(path))
    pfx = "orf_" if prec == "f32" else "ord_"
    vp, i64, P = C.c_void_p, C.c_longlong, C.POINTER
    real = C.c_float if prec == "f32" else C.c_double

    def sig(name, res, args):
        fn = getattr(lib, pfx + name)
        fn.restype = res
        fn.argtypes = args

    sig("kernel_root", C.c_float, [])
    sig("kernel_norm", C.c_float, [])
    sig("kernel_gamma", C.c_float, [])
    sig("kernel_deval", None, [real, P(real), P(real)])
    for n in ("box_density", "box_gradient", "box_force"):
        sig(n, i64, [vp, i64, P(abi.HydroParams), vp])
    sig("box_density_subset", i64, [vp, i64, P(abi.HydroParams), vp, i64])
    sig("init_parts", None, [vp, i64, P(abi.HydroParams)])
    sig("box_ghost", C.c_int, [vp, i64, P(abi.HydroParams), P(i64)])
    sig("box_extra_ghost", None, [vp, i64, P(abi.HydroParams)])
    sig("box_end_force", None, [vp, i64, P(abi.HydroParams)])
    sig("box_drift", None, [vp, vp, vp, i64, P(abi.DriftParams)])
    sig("box_count_pairs", i64, [vp, i64, P(abi.HydroParams), C.c_int])
    sig("grav_self_pp", i64, [vp, C.c_int, P(C.c_double), P(C.c_double), C.c_double,
                              P(abi.GravParams)])
    sig("grav_pair_pp", i64, [vp, C.c_int, vp, C.c_int, P(C.c_double), P(C.c_double),
                              C.c_double, C.c_double, C.c_int, P(abi.GravParams)])
    sig("grav_pp_leaves", i64, [vp, vp, C.c_int, vp, vp, P(abi.GravParams), vp, P(i64)])
    sig("grav_pair_pp_mpole", i64, [vp, C.c_int, vp, C.c_int, P(abi.Multipole),
                                    P(abi.Multipole), C.c_int, C.c_int, P(abi.GravParams),
                                    P(i64)])
    sig("grav_p2m", None, [vp, C.c_int, P(abi.Multipole)])
    sig("grav_m2m", None, [vp, C.c_int, P(C.c_double), P(C.c_double), P(abi.Multipole)])
    sig("grav_tree", None, [vp, C.c_int, vp, C.c_int, vp, C.c_int, vp, C.c_int,
                            P(abi.GravParams), vp, vp])
    sig("grav_tree_owned", None, [vp, C.c_int, vp, C.c_int, vp, C.c_int, vp, C.c_int,
                                  P(abi.GravParams), vp, vp, vp])
    sig("grav_m2l_pairs", None, [P(abi.GravParams), vp, C.c_int, vp, C.c_int, vp])
    sig("grav_m2l_accept_symmetric", C.c_int, [P(abi.GravParams), P(abi.Multipole),
                                               P(abi.Multipole), C.c_double])
    sig("pm_mesh", None, [vp, C.c_int, C.c_int, C.c_double, C.c_double, C.c_float, vp])
    if prec == "f32":
        for n in ("iact_density", "iact_force", "iact_gradient"):
            sig(n, None, [real, P(real), real, real, vp, vp, real, real])
        for n in ("iact_nonsym_density", "iact_nonsym_force", "iact_nonsym_gradient"):
            sig(n, None, [real, P(real), real, real, vp, vp, real, real])
        sig("cell_sort", None, [vp, C.c_int])
        sig("cell_free_sorts", None, [vp])
        for n in ("dopair1_branch",):
            sig(n, C.c_int, [vp, vp, vp, C.c_int])
        sig("doself1_branch", C.c_int, [vp, vp, C.c_int])
        sig("dopair2_branch", C.c_int, [vp, vp, vp])
        sig("doself2_branch", C.c_int, [vp, vp])
        sig("doself_subset", None, [vp, vp, vp, P(C.c_int), C.c_int])
        sig("dopair_subset", None, [vp, vp, vp, P(C.c_int), C.c_int, vp])
        for n in ("pairs_all_density", "pairs_all_force"):
            sig(n, None, [vp, vp, vp])
        for n in ("self_all_density", "self_all_force"):
            sig(n, None, [vp, vp])
        for n in ("part_end_density", "part_prepare_gradient", "part_extra_ghost"):
            sig(n, None, [vp, P(abi.HydroParams)])
        sig("part_end_force", None, [vp])
        sig("part_init", None, [vp])
        sig("cellgrid_new", vp, [vp, i64, C.c_double, C.c_int])
        sig("cellgrid_free", None, [vp])
        sig("cellgrid_parts", vp, [vp])
        sig("cellgrid_run", C.c_double, [vp, vp, C.c_int, C.c_int])
        sig("celltree_new", vp, [vp, i64, C.c_double, C.c_int, C.c_int])
        sig("celltree_free", None, [vp])
        sig("celltree_parts", vp, [vp])
        sig("celltree_ncells", i64, [vp])
        sig("celltree_run", C.c_double, [vp, vp, C.c_int, C.c_int])
    lib.pfx = pfx
    _libs[key] = lib
    return lib


def fn(prec: str, name: str, kernel: str = "cubic-spline"):
    lib = load(prec, kernel)
    return getattr(lib, lib.pfx + name)


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class CellSet:
    """A set of SWIFT-style cells over one contiguous part array (the way
    test27cells/test125cells build their cells), usable by both the oracle's
    sorted loops and the SWIFT-signature adapter."""

    def __init__(self, parts: np.ndarray, bounds, locs, width, ti=8):
        self.parts = parts
        self.cells = (abi.Cell * len(bounds))()
        for c, ((s, e), loc) in enumerate(zip(bounds, locs)):
            cell = self.cells[c]
            for k in range(3):
                cell.loc[k] = loc[k]
                cell.width[k] = width
            cell.dmin = width
            sub = parts[s:e]
            cell.hydro.parts = parts.ctypes.data + s * parts.itemsize
            cell.hydro.count = e - s
            hmax = float(sub["h"].max()) if e > s else 0.0
            cell.hydro.h_max = cell.hydro.h_max_old = cell.hydro.h_max_active = hmax
            cell.hydro.ti_end_min = ti
            cell.hydro.ti_old_part = ti
            cell.grav.ti_end_min = ti
        self.bounds = list(bounds)

    def ptr(self, c: int) -> int:
        return C.addressof(self.cells[c])

    def sort_all(self):
        f = fn("f32", "cell_sort")
        for c in range(len(self.cells)):
            f(self.ptr(c), 0x1FFF)

    def free_sorts(self):
        f = fn("f32", "cell_free_sorts")
        for c in range(len(self.cells)):
            f(self.ptr(c))

    def view(self, c: int) -> np.ndarray:
        s, e = self.bounds[c]
        return self.parts[s:e]
