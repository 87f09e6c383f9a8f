"""ctypes bindings of libswifthip (include/swifthip.h) and the SWIFT-signature
adapter (include/swifthip_swift.h).

The product path is the HIP library: if ``libswifthip.so`` is missing this
module raises immediately — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

from . import abi

PKG = Path(__file__).resolve().parent
# SWH_LIB_PATH: developer override (occupancy experiments, tools/build_variant.sh)
LIB_PATH = Path(os.environ.get("SWH_LIB_PATH", str(PKG / "libswifthip.so")))
ADAPTER_PATH = PKG / "libswifthip_swift.so"
# The SPH kernel is a build-time choice, as SWIFT's configure --with-kernel
# (configure.ac:2107-2137): one library per kernel, the same C ABI.
KERNEL_LIBS = {"cubic-spline": LIB_PATH, "wendland-c2": PKG / "libswifthip_wc2.so"}
ADAPTER_LIBS = {"cubic-spline": ADAPTER_PATH, "wendland-c2": PKG / "libswifthip_swift_wc2.so"}

STATUS = {
    0: "ok", 1: "invalid argument", 2: "HIP runtime error", 3: "Interacting unsorted cells.",
    4: "Cell smaller than smoothing length", 5: "Smoothing length failed to converge",
    6: "no usable gfx950 device", 7: "device out of memory", 8: "call out of order",
}

# Every symbol include/swifthip.h declares (checked by tests/test_abi.py).
HIP_SYMBOLS = [
    "swh_part_layout_sphenix", "swh_gpart_layout_multisoftening", "swh_init", "swh_finalize",
    "swh_set_precision", "swh_status_string", "swh_last_error", "swh_abi_version",
    "swh_kernel_name",
    "swh_doself_density", "swh_dopair_density", "swh_doself_gradient", "swh_dopair_gradient",
    "swh_doself_force", "swh_dopair_force", "swh_doself_subset_density",
    "swh_dopair_subset_density", "swh_grav_self_pp", "swh_grav_pair_pp", "swh_space_create",
    "swh_space_destroy", "swh_space_set_stream", "swh_space_upload_parts",
    "swh_space_download_parts", "swh_space_count", "swh_space_rebuild", "swh_space_init_parts",
    "swh_space_reset_acceleration",
    "swh_density_loop", "swh_ghost", "swh_gradient_loop", "swh_extra_ghost", "swh_force_loop",
    "swh_end_force", "swh_space_sync", "swh_space_query", "swh_space_set_tuning", "swh_space_get_info",
    "swh_space_set_owned", "swh_space_pack_halo", "swh_space_unpack_halo",
    "swh_gspace_create",
    "swh_gspace_destroy", "swh_gspace_upload", "swh_gspace_set_leaves", "swh_grav_pp_batch",
    "swh_gspace_make_multipoles", "swh_space_upload_xparts", "swh_space_drift",
    "swh_gspace_set_tree", "swh_gspace_set_owned_cells", "swh_grav_tree",
    "swh_grav_tree_tasks", "swh_gspace_field_tensors", "swh_gspace_multipoles",
    "swh_gspace_set_multipoles", "swh_gspace_grav_down",
    "swh_gspace_download", "swh_gspace_sync", "swh_gspace_query", "swh_gspace_pm_mesh",
    "swh_grav_m2l_pairs", "swh_grav_m2l_accept",
]
ADAPTER_SYMBOLS = [
    "swifthip_swift_init", "swifthip_swift_finalize", "swifthip_swift_last_error",
    "swifthip_swift_set_precision",
    "swifthip_swift_clear_error", "runner_doself1_branch_density",
    "runner_dopair1_branch_density", "runner_doself1_branch_gradient",
    "runner_dopair1_branch_gradient", "runner_doself2_branch_force",
    "runner_dopair2_branch_force", "runner_doself_subset_branch_density",
    "runner_dopair_subset_branch_density", "runner_doself_grav_pp", "runner_dopair_grav_pp",
    "runner_doself_recursive_grav", "runner_dopair_recursive_grav", "runner_do_grav_down",
    "runner_dosub_self1_density", "runner_dosub_pair1_density", "runner_dosub_self1_gradient",
    "runner_dosub_pair1_gradient", "runner_dosub_self2_force", "runner_dosub_pair2_force",
    "runner_dosub_subset_density", "swifthip_swift_part_layout", "swifthip_swift_gpart_layout",
    "swifthip_swift_split_pairs", "runner_dopair_grav_mm_progenies", "runner_do_grav_long_range",
]


class SwhError(RuntimeError):
    def __init__(self, status: int, where: str, detail: str = ""):
        self.status = status
        super().__init__(f"{where}: {STATUS.get(status, status)} {detail}".strip())


_libs: dict = {}
_adapters: dict = {}



SWH_BUSY = 9  # swh_*_query: queued work still running

def load(kernel: str = "cubic-spline") -> C.CDLL:
    """Load the libswifthip built for `kernel` (raises if it was not built).
    Every kernel's library is private to its handle (RTLD_LOCAL): the
    libraries export the same swh_* names, and a global one would capture the
    other adapter's calls (global scope is searched before a library's own
    dependencies)."""
    if kernel in _libs:
        return _libs[kernel]
    if kernel not in KERNEL_LIBS:
        raise ValueError(f"unknown SPH kernel {kernel!r}: {sorted(KERNEL_LIBS)}")
    path = KERNEL_LIBS[kernel]
    if not path.exists():
        raise ImportError(
            f"{path} is missing: build it with `python -m swift_subtask_dev_amd.build` "
            "(the HIP library is the only implementation of this path)")
    lib = C.CDLL(str(path), mode=C.RTLD_LOCAL)
    vp, i32, i64, dp = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    P = C.POINTER
    sigs = {
        "swh_part_layout_sphenix": (None, [P(abi.PartLayout)]),
        "swh_gpart_layout_multisoftening": (None, [P(abi.GPartLayout)]),
        "swh_init": (C.c_int, [P(vp), C.c_int]),
        "swh_finalize": (C.c_int, [vp]),
        "swh_set_precision": (C.c_int, [vp, C.c_int]),
        "swh_status_string": (C.c_char_p, [C.c_int]),
        "swh_last_error": (C.c_char_p, []),
        "swh_abi_version": (C.c_int, []),
        "swh_kernel_name": (C.c_char_p, []),
        "swh_doself_density": (C.c_int, [vp, P(abi.CellView), P(abi.PartLayout), P(abi.HydroParams)]),
        "swh_doself_gradient": (C.c_int, [vp, P(abi.CellView), P(abi.PartLayout), P(abi.HydroParams)]),
        "swh_doself_force": (C.c_int, [vp, P(abi.CellView), P(abi.PartLayout), P(abi.HydroParams)]),
        "swh_dopair_density": (C.c_int, [vp, P(abi.CellView), P(abi.CellView), P(dp), P(abi.PartLayout), P(abi.HydroParams)]),
        "swh_dopair_gradient": (C.c_int, [vp, P(abi.CellView), P(abi.CellView), P(dp), P(abi.PartLayout), P(abi.HydroParams)]),
        "swh_dopair_force": (C.c_int, [vp, P(abi.CellView), P(abi.CellView), P(dp), P(abi.PartLayout), P(abi.HydroParams)]),
        "swh_doself_subset_density": (C.c_int, [vp, P(abi.CellView), vp, P(i32), i32, P(abi.PartLayout), P(abi.HydroParams)]),
        "swh_dopair_subset_density": (C.c_int, [vp, P(abi.CellView), vp, P(i32), i32, P(abi.CellView), P(dp), P(abi.PartLayout), P(abi.HydroParams)]),
        "swh_grav_self_pp": (C.c_int, [vp, P(abi.GCellView), P(abi.GPartLayout), P(abi.GravParams)]),
        "swh_grav_pair_pp": (C.c_int, [vp, P(abi.GCellView), P(abi.GCellView), C.c_int, C.c_int, P(abi.GPartLayout), P(abi.GravParams)]),
        "swh_space_create": (C.c_int, [vp, P(vp)]),
        "swh_space_destroy": (C.c_int, [vp]),
        "swh_space_set_stream": (C.c_int, [vp, vp]),
        "swh_space_upload_parts": (C.c_int, [vp, vp, i64, P(abi.PartLayout), C.c_int]),
        "swh_space_download_parts": (C.c_int, [vp, vp, P(abi.PartLayout), C.c_int, C.c_int]),
        "swh_space_count": (i64, [vp]),
        "swh_space_rebuild": (C.c_int, [vp, P(abi.HydroParams), dp]),
        "swh_space_init_parts": (C.c_int, [vp, P(abi.HydroParams)]),
        "swh_space_reset_acceleration": (C.c_int, [vp, P(abi.HydroParams)]),
        "swh_density_loop": (C.c_int, [vp, P(abi.HydroParams), P(i64)]),
        "swh_ghost": (C.c_int, [vp, P(abi.HydroParams), P(i32), P(i64)]),
        "swh_gradient_loop": (C.c_int, [vp, P(abi.HydroParams), P(i64)]),
        "swh_extra_ghost": (C.c_int, [vp, P(abi.HydroParams)]),
        "swh_force_loop": (C.c_int, [vp, P(abi.HydroParams), P(i64)]),
        "swh_end_force": (C.c_int, [vp, P(abi.HydroParams)]),
        "swh_space_sync": (C.c_int, [vp]),
        "swh_space_query": (C.c_int, [vp]),
        "swh_space_set_owned": (C.c_int, [vp, i64]),
        "swh_space_pack_halo": (C.c_int, [vp, vp, i32, vp]),
        "swh_space_unpack_halo": (C.c_int, [vp, vp, i32, vp, C.c_int]),
        "swh_space_upload_xparts": (C.c_int, [vp, vp, i64, P(abi.XPartLayout), C.c_int]),
        "swh_space_drift": (C.c_int, [vp, P(abi.DriftParams), P(abi.HydroParams)]),
        "swh_space_set_tuning": (C.c_int, [vp, P(abi.Tuning)]),
        "swh_space_get_info": (C.c_int, [vp, P(abi.SpaceInfo)]),
        "swh_gspace_create": (C.c_int, [vp, P(vp)]),
        "swh_gspace_destroy": (C.c_int, [vp]),
        "swh_gspace_upload": (C.c_int, [vp, vp, i64, P(abi.GPartLayout), C.c_int]),
        "swh_gspace_set_leaves": (C.c_int, [vp, vp, i32, P(i32), vp, i32]),
        "swh_grav_pp_batch": (C.c_int, [vp, P(abi.GravParams), P(i64), P(i64)]),
        "swh_gspace_make_multipoles": (C.c_int, [vp, vp]),
        "swh_gspace_set_tree": (C.c_int, [vp, vp, i32]),
        "swh_gspace_set_owned_cells": (C.c_int, [vp, P(C.c_uint8), i32]),
        "swh_grav_tree": (C.c_int, [vp, P(abi.GravParams), vp, i32, vp, i32,
                                    P(abi.GravTreeStats)]),
        "swh_gspace_field_tensors": (C.c_int, [vp, vp]),
        "swh_grav_tree_tasks": (C.c_int, [vp, P(abi.GravParams), vp, i32, vp, i32, i32,
                                          P(abi.GravTreeStats)]),
        "swh_gspace_multipoles": (C.c_int, [vp, vp]),
        "swh_gspace_set_multipoles": (C.c_int, [vp, vp]),
        "swh_gspace_grav_down": (C.c_int, [vp, P(abi.GravParams), vp]),
        "swh_gspace_download": (C.c_int, [vp, vp, P(abi.GPartLayout), C.c_int]),
        "swh_gspace_sync": (C.c_int, [vp]),
        "swh_gspace_query": (C.c_int, [vp]),
        "swh_gspace_pm_mesh": (C.c_int, [vp, P(abi.PMParams), vp]),
        "swh_grav_m2l_pairs": (C.c_int, [vp, P(abi.GravParams), vp, i32, vp, i32, vp]),
        "swh_grav_m2l_accept": (C.c_int, [P(abi.GravParams), P(abi.Multipole),
                                          P(abi.Multipole), dp]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    ver = lib.swh_abi_version()
    if ver != abi.ABI_VERSION:
        # a struct such as swh_grav_tree_stats grew between versions: a mismatched
        # library would write past (or leave unset) the ctypes layouts' fields
        raise ImportError(f"{path} has C ABI v{ver}; these bindings are written for "
                          f"v{abi.ABI_VERSION} (rebuild it)")
    got = lib.swh_kernel_name().decode()
    if got != kernel:
        raise ImportError(f"{path} was built for the {got} kernel, not {kernel}")
    _libs[kernel] = lib
    return lib


def load_adapter(kernel: str = "cubic-spline") -> C.CDLL:
    if kernel in _adapters:
        return _adapters[kernel]
    if "SWH_LIB_PATH" in os.environ and kernel == "cubic-spline":
        # the adapter links its own $ORIGIN/libswifthip.so: with an override
        # the process would hold two copies (two contexts, two error states)
        # and the adapter tests would silently run the in-tree build
        raise ImportError("SWH_LIB_PATH overrides libswifthip.so, but the SWIFT-signature "
                          "adapter is linked against the in-tree build: unset SWH_LIB_PATH "
                          "to load the adapter")
    load(kernel)
    path = ADAPTER_LIBS[kernel]
    if not path.exists():
        raise ImportError(f"{path} is missing: run the build")
    ad = C.CDLL(str(path))
    vp, P = C.c_void_p, C.POINTER
    ad.swifthip_swift_init.restype = C.c_int
    ad.swifthip_swift_init.argtypes = [C.c_int, C.c_int]
    ad.swifthip_swift_finalize.restype = None
    ad.swifthip_swift_set_precision.restype = C.c_int
    ad.swifthip_swift_set_precision.argtypes = [C.c_int]
    ad.swifthip_swift_last_error.restype = C.c_char_p
    ad.swifthip_swift_clear_error.restype = None
    for n in ("runner_doself1_branch_density", "runner_doself1_branch_gradient",
              "runner_doself2_branch_force", "runner_doself_grav_pp"):
        getattr(ad, n).argtypes = [vp, vp]
        getattr(ad, n).restype = None
    for n in ("runner_dopair1_branch_density", "runner_dopair1_branch_gradient",
              "runner_dopair2_branch_force"):
        getattr(ad, n).argtypes = [vp, vp, vp]
        getattr(ad, n).restype = None
    ad.runner_doself_subset_branch_density.argtypes = [vp, vp, vp, P(C.c_int), C.c_int]
    ad.runner_doself_subset_branch_density.restype = None
    ad.runner_dopair_subset_branch_density.argtypes = [vp, vp, vp, P(C.c_int), C.c_int, vp]
    ad.runner_dopair_subset_branch_density.restype = None
    ad.runner_dopair_grav_pp.argtypes = [vp, vp, vp, C.c_int, C.c_int]
    ad.runner_dopair_grav_pp.restype = None
    for n in ("runner_doself_recursive_grav", "runner_do_grav_down"):
        getattr(ad, n).argtypes = [vp, vp, C.c_int]
        getattr(ad, n).restype = None
    ad.runner_dopair_recursive_grav.argtypes = [vp, vp, vp, C.c_int]
    ad.runner_dopair_recursive_grav.restype = None
    ad.runner_dopair_grav_mm_progenies.argtypes = [vp, C.c_longlong, vp, vp]
    ad.runner_dopair_grav_mm_progenies.restype = None
    ad.runner_do_grav_long_range.argtypes = [vp, vp, C.c_int]
    ad.runner_do_grav_long_range.restype = None
    _adapters[kernel] = ad
    return ad


def _check(status: int, where: str, lib: C.CDLL | None = None) -> None:
    if status != 0:
        detail = ((lib or load()).swh_last_error() or b"").decode(errors="replace")
        raise SwhError(status, where, detail)


def part_layout() -> abi.PartLayout:
    L = abi.PartLayout()
    load().swh_part_layout_sphenix(C.byref(L))
    return L


def gpart_layout() -> abi.GPartLayout:
    L = abi.GPartLayout()
    load().swh_gpart_layout_multisoftening(C.byref(L))
    return L


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class Context:
    """One swh_context (device + per-task streams)."""

    def __init__(self, device: int = 0, precision: str = "f64", kernel: str = "cubic-spline"):
        lib = load(kernel)
        self.kernel = kernel
        self._lib = lib
        h = C.c_void_p()
        _check(lib.swh_init(C.byref(h), device), "swh_init", self._lib)
        self.handle = h
        self.set_precision(precision)
        self.L = part_layout()
        self.GL = gpart_layout()

    def set_precision(self, precision: str) -> None:
        _check(self._lib.swh_set_precision(self.handle, 0 if precision == "f64" else 1),
               "swh_set_precision", self._lib)
        self.precision = precision

    def close(self) -> None:
        if self.handle:
            self._lib.swh_finalize(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- per-task -------------------------------------------------------
    def cell_view(self, parts: np.ndarray, loc, width, active=True) -> abi.CellView:
        v = abi.CellView()
        v.parts = _ptr(parts)
        v.count = len(parts)
        v.active = 1 if active else 0
        for k in range(3):
            v.loc[k] = loc[k]
            v.width[k] = width[k]
        return v

    def doself(self, loop: str, view: abi.CellView, P: abi.HydroParams) -> None:
        fn = {"density": self._lib.swh_doself_density, "gradient": self._lib.swh_doself_gradient,
              "force": self._lib.swh_doself_force}[loop]
        _check(fn(self.handle, C.byref(view), C.byref(self.L), C.byref(P)), f"doself_{loop}", self._lib)

    def dopair(self, loop: str, vi, vj, shift, P) -> None:
        fn = {"density": self._lib.swh_dopair_density, "gradient": self._lib.swh_dopair_gradient,
              "force": self._lib.swh_dopair_force}[loop]
        sh = (C.c_double * 3)(*shift)
        _check(fn(self.handle, C.byref(vi), C.byref(vj), sh, C.byref(self.L), C.byref(P)),
               f"dopair_{loop}", self._lib)


class HydroSpace:
    """Device-resident particle set (swh_space): the batch loops."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self._lib = ctx._lib
        h = C.c_void_p()
        _check(self._lib.swh_space_create(ctx.handle, C.byref(h)), "swh_space_create", self._lib)
        self.handle = h

    def close(self):
        if self.handle:
            self._lib.swh_space_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_tuning(self, cell_factor=1, loop_variant=0, group_size=0, cell_scale=0.0,
                   diag_mode=0, list_capacity=0, list_skin=abi.DEFAULT_LIST_SKIN, list_keep=0):
        t = abi.Tuning(cell_factor, loop_variant, group_size, cell_scale, diag_mode,
                       list_capacity, list_skin, list_keep)
        _check(self._lib.swh_space_set_tuning(self.handle, C.byref(t)), "set_tuning", self._lib)

    def info(self) -> dict:
        i = abi.SpaceInfo()
        _check(self._lib.swh_space_get_info(self.handle, C.byref(i)), "get_info", self._lib)
        return {"cdim": list(i.cdim), "ncell": i.ncell, "ngroups": i.ngroups,
                "cell_width": list(i.cell_width), "h_max": i.h_max,
                "loop_stats": list(i.loop_stats), "list_entries": i.list_entries,
                "list_overflow": i.list_overflow, "list_valid": bool(i.list_valid),
                "dx_max": i.dx_max, "list_builds": i.list_builds}

    def upload(self, parts, count=None, on_device=False):
        """parts: numpy PART_DTYPE array (host) or a device pointer (int) with count."""
        if on_device:
            _check(self._lib.swh_space_upload_parts(self.handle, C.c_void_p(parts), count,
                                                    C.byref(self.ctx.L), 1), "upload", self._lib)
        else:
            _check(self._lib.swh_space_upload_parts(self.handle, _ptr(parts), len(parts),
                                                    C.byref(self.ctx.L), 0), "upload", self._lib)

    def download(self, parts: np.ndarray, fields=abi.FIELDS_ALL):
        _check(self._lib.swh_space_download_parts(self.handle, _ptr(parts), C.byref(self.ctx.L),
                                                  fields, 0), "download", self._lib)

    def rebuild(self, P, min_cell_width=0.0):
        _check(self._lib.swh_space_rebuild(self.handle, C.byref(P), min_cell_width), "rebuild", self._lib)

    def init_parts(self, P):
        _check(self._lib.swh_space_init_parts(self.handle, C.byref(P)), "init_parts", self._lib)

    def reset_acceleration(self, P):
        _check(self._lib.swh_space_reset_acceleration(self.handle, C.byref(P)),
               "reset_acceleration", self._lib)

    def set_stream(self, stream_ptr: int):
        """Bind a HIP stream (e.g. torch.cuda.current_stream().cuda_stream)."""
        _check(self._lib.swh_space_set_stream(self.handle, C.c_void_p(stream_ptr)), "set_stream", self._lib)

    def _loop(self, fn, P, count):
        n = C.c_int64(0)
        _check(fn(self.handle, C.byref(P), C.byref(n) if count else None), fn.__name__, self._lib)
        return n.value if count else None

    def density(self, P, count=True):
        return self._loop(self._lib.swh_density_loop, P, count)

    def gradient(self, P, count=True):
        return self._loop(self._lib.swh_gradient_loop, P, count)

    def force(self, P, count=True):
        return self._loop(self._lib.swh_force_loop, P, count)

    def ghost(self, P):
        it = C.c_int32(0)
        nu = C.c_int64(0)
        _check(self._lib.swh_ghost(self.handle, C.byref(P), C.byref(it), C.byref(nu)), "ghost", self._lib)
        return it.value, nu.value

    def extra_ghost(self, P):
        _check(self._lib.swh_extra_ghost(self.handle, C.byref(P)), "extra_ghost", self._lib)

    def end_force(self, P):
        _check(self._lib.swh_end_force(self.handle, C.byref(P)), "end_force", self._lib)

    def sync(self):
        _check(self._lib.swh_space_sync(self.handle), "sync", self._lib)

    def done(self) -> bool:
        """swh_space_query: True once the queued work has finished (no wait)."""
        r = self._lib.swh_space_query(self.handle)
        if r == SWH_BUSY:
            return False
        _check(r, "query", self._lib)
        return True

    def upload_xparts(self, xparts: np.ndarray):
        """struct xpart array (abi.XPART_DTYPE), same order/count as the parts."""
        XL = abi.XPartLayout(abi.XPART_DTYPE.itemsize, abi.XPART_DTYPE.fields["v_full"][1],
                             abi.XPART_DTYPE.fields["a_grav"][1])
        _check(self._lib.swh_space_upload_xparts(self.handle, _ptr(xparts), len(xparts),
                                                 C.byref(XL), 0), "upload_xparts", self._lib)

    def drift(self, D: abi.DriftParams, P: abi.HydroParams):
        _check(self._lib.swh_space_drift(self.handle, C.byref(D), C.byref(P)), "drift", self._lib)

    def set_owned(self, n_owned: int):
        """Caller indices >= n_owned become read-only halo (foreign) particles."""
        _check(self._lib.swh_space_set_owned(self.handle, n_owned), "set_owned", self._lib)

    def pack_halo(self, idx_ptr: int, n: int, out_ptr: int):
        """Device pointers: int32 caller indices -> n * 8 float halo records."""
        _check(self._lib.swh_space_pack_halo(self.handle, C.c_void_p(idx_ptr), n,
                                             C.c_void_p(out_ptr)), "pack_halo", self._lib)

    def unpack_halo(self, idx_ptr: int, n: int, in_ptr: int, fields: int = 31):
        _check(self._lib.swh_space_unpack_halo(self.handle, C.c_void_p(idx_ptr), n,
                                               C.c_void_p(in_ptr), fields), "unpack_halo", self._lib)

    def hydro_step(self, P):
        """The full SPHENIX hydro chain of one step:
        density -> ghost -> gradient -> extra ghost -> force -> end force."""
        self.init_parts(P)
        nd = self.density(P)
        it, _ = self.ghost(P)
        ng = self.gradient(P)
        self.extra_ghost(P)
        nf = self.force(P)
        self.end_force(P)
        return {"density": nd, "gradient": ng, "force": nf, "ghost_iterations": it}


class GravSpace:
    """Device-resident gpart set for batch P2P (swh_gspace)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self._lib = ctx._lib
        h = C.c_void_p()
        _check(self._lib.swh_gspace_create(ctx.handle, C.byref(h)), "swh_gspace_create", self._lib)
        self.handle = h

    def close(self):
        if self.handle:
            self._lib.swh_gspace_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, gparts: np.ndarray):
        _check(self._lib.swh_gspace_upload(self.handle, _ptr(gparts), len(gparts),
                                           C.byref(self.ctx.GL), 0), "gspace_upload", self._lib)

    def set_leaves(self, leaves: np.ndarray, pair_offset: np.ndarray, pairs: np.ndarray):
        leaves = np.ascontiguousarray(leaves, dtype=abi.LEAF_DTYPE)
        pair_offset = np.ascontiguousarray(pair_offset, dtype=np.int32)
        pairs = np.ascontiguousarray(pairs, dtype=abi.LEAF_PAIR_DTYPE)
        self._keep = (leaves, pair_offset, pairs)
        _check(self._lib.swh_gspace_set_leaves(
            self.handle, _ptr(leaves), len(leaves),
            pair_offset.ctypes.data_as(C.POINTER(C.c_int32)), _ptr(pairs), len(pairs)),
            "set_leaves", self._lib)

    def make_multipoles(self, want=False):
        """Leaf multipoles on the device (P2M); want=True returns a host copy
        (ctypes array of abi.Multipole)."""
        out = (abi.Multipole * max(1, len(self._keep[0])))() if want else None
        _check(self._lib.swh_gspace_make_multipoles(self.handle, out), "make_multipoles", self._lib)
        return out

    def pp(self, G: abi.GravParams, count=True, m2p=False):
        """P2P (+ M2P on allow_mpole pairs). count: P2P interactions; with
        m2p=True returns (P2P interactions, M2P evaluations)."""
        n, m = C.c_int64(0), C.c_int64(0)
        _check(self._lib.swh_grav_pp_batch(self.handle, C.byref(G), C.byref(n) if count else None,
                                           C.byref(m) if m2p else None), "grav_pp_batch", self._lib)
        if m2p:
            return n.value, m.value
        return n.value if count else None

    def set_tree(self, cells: np.ndarray):
        """cells: records of (start, count, split, progeny[8]) (ics.gravity_tree)."""
        cells = np.ascontiguousarray(cells)
        assert cells.dtype.itemsize == C.sizeof(abi.GCell)
        self._tree = cells
        _check(self._lib.swh_gspace_set_tree(self.handle, _ptr(cells), len(cells)), "set_tree", self._lib)

    def set_owned_cells(self, owned):
        """Per-cell ownership (uint8, whole subtrees; None: every cell) for a
        step sharded over ranks (swh_gspace_set_owned_cells)."""
        if owned is None:
            _check(self._lib.swh_gspace_set_owned_cells(self.handle, None, 0), "set_owned_cells", self._lib)
            return
        owned = np.ascontiguousarray(owned, dtype=np.uint8)
        self._owned = owned
        _check(self._lib.swh_gspace_set_owned_cells(
            self.handle, owned.ctypes.data_as(C.POINTER(C.c_uint8)), len(owned)),
            "set_owned_cells", self._lib)

    def tree(self, G: abi.GravParams, self_cells, pair_cells, stats: bool = True) -> dict:
        """runner_doself_recursive_grav on self_cells, runner_dopair_recursive_grav
        on pair_cells (n x 2), then the down pass. stats=False: no phase
        events and no counting pass (returns None)."""
        sc = np.ascontiguousarray(self_cells, dtype=np.int32)
        pc = np.ascontiguousarray(pair_cells, dtype=np.int32).reshape(-1)
        st = abi.GravTreeStats()
        _check(self._lib.swh_grav_tree(self.handle, C.byref(G), _ptr(sc), len(sc), _ptr(pc),
                                       len(pc) // 2, C.byref(st) if stats else None),
               "grav_tree", self._lib)
        if not stats:
            return None
        return {"n_pp": st.n_pp, "n_m2p": st.n_m2p, "n_m2l": st.n_m2l,
                "n_pp_tasks": st.n_pp_tasks, "n_skipped": st.n_skipped,
                "n_pp_truncated": st.n_pp_truncated,
                "ms": {"multipoles": st.ms_multipoles, "walk": st.ms_walk, "p2p": st.ms_p2p,
                       "m2p": st.ms_m2p, "down": st.ms_down}}

    def multipoles(self):
        """The tree cells' multipoles (abi.Multipole array)."""
        out = (abi.Multipole * len(self._tree))()
        _check(self._lib.swh_gspace_multipoles(self.handle, out), "multipoles", self._lib)
        return out

    def field_tensors(self) -> np.ndarray:
        out = np.zeros((len(self._tree), abi.MPOLE_TERMS), dtype=np.float32)
        _check(self._lib.swh_gspace_field_tensors(self.handle, _ptr(out)), "field_tensors", self._lib)
        return out

    def download(self, gparts: np.ndarray):
        _check(self._lib.swh_gspace_download(self.handle, _ptr(gparts), C.byref(self.ctx.GL), 0),
               "gspace_download", self._lib)

    def sync(self):
        _check(self._lib.swh_gspace_sync(self.handle), "gspace_sync", self._lib)

    def done(self) -> bool:
        """swh_gspace_query: True once the queued work has finished (no wait)."""
        r = self._lib.swh_gspace_query(self.handle)
        if r == SWH_BUSY:
            return False
        _check(r, "gspace_query", self._lib)
        return True

    def pm_mesh(self, N: int, box_size: float, r_s: float, const_G: float = 1.0,
                want_potential: bool = False):
        """PM long-range gravity (swh_gspace_pm_mesh): the records' a_grav_mesh /
        potential_mesh are set on the device (download returns them); returns
        the N^3 potential mesh if asked."""
        M = abi.PMParams(N, abi.GPART_OFF_A_GRAV_MESH, abi.GPART_OFF_POTENTIAL_MESH, 0,
                         box_size, r_s, const_G)
        pot = np.zeros((N, N, N), dtype=np.float64) if want_potential else None
        _check(self._lib.swh_gspace_pm_mesh(self.handle, C.byref(M),
                                            _ptr(pot) if pot is not None else None), "pm_mesh", self._lib)
        return pot
