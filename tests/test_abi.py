"""CPU checks of the C-ABI boundary: the libraries load without a GPU and
export every symbol the public headers declare; the Python layout mirrors
match the C structs."""
from __future__ import annotations

import ctypes as C
import re
from pathlib import Path

import numpy as np

from swift_subtask_dev_amd import abi, lib

INCLUDE = Path(__file__).resolve().parents[1] / "include"


def _declared(header: str, macro: str):
    text = (INCLUDE / header).read_text()
    names = set(re.findall(macro + r"\s+[\w\s\*]*?\b(\w+)\s*\(", text))
    return sorted(n for n in names if not n.startswith("__"))


def test_hip_library_exports_header():
    L = lib.load()
    declared = _declared("swifthip.h", "SWH_API")
    assert len(declared) >= 40
    assert sorted(declared) == sorted(lib.HIP_SYMBOLS)
    for name in declared:
        assert hasattr(L, name), name


def test_adapter_exports_header():
    ad = lib.load_adapter()
    declared = _declared("swifthip_swift.h", "SWHS_API")
    assert sorted(declared) == sorted(lib.ADAPTER_SYMBOLS)
    for name in declared:
        assert hasattr(ad, name), name


def test_no_device_reports_cleanly():
    """Without a GPU, swh_init fails with a status code, never aborts."""
    L = lib.load()
    h = C.c_void_p()
    import torch

    if torch.cuda.is_available():
        return
    st = L.swh_init(C.byref(h), 0)
    assert st == 6  # SWH_ERR_NO_DEVICE
    assert L.swh_status_string(st) == b"no usable gfx950 device"


def test_part_layout_matches_dtype():
    Lp = lib.part_layout()
    assert Lp.stride == 160 == abi.PART_DTYPE.itemsize
    f = abi.PART_DTYPE.fields
    pairs = {"off_id": "id", "off_x": "x", "off_v": "v", "off_a_hydro": "a_hydro",
             "off_mass": "mass", "off_h": "h", "off_u": "u", "off_u_dt": "u_dt",
             "off_rho": "rho", "off_div_v": "div_v", "off_div_v_dt": "div_v_dt",
             "off_div_v_previous_step": "div_v_previous_step", "off_visc_alpha": "visc_alpha",
             "off_v_sig": "v_sig", "off_laplace_u": "laplace_u", "off_diff_alpha": "diff_alpha",
             "off_wcount": "wcount", "off_wcount_dh": "wcount_dh", "off_rho_dh": "rho_dh",
             "off_rot_v": "rot_v", "off_f": "f", "off_pressure": "pressure",
             "off_soundspeed": "soundspeed", "off_h_dt": "h_dt", "off_balsara": "balsara",
             "off_alpha_visc_max_ngb": "alpha_visc_max_ngb", "off_time_bin": "time_bin",
             "off_min_ngb_time_bin": "min_ngb_time_bin"}
    for off, name in pairs.items():
        assert getattr(Lp, off) == f[name][1], (off, name)
    G = lib.gpart_layout()
    assert G.stride == 96 == abi.GPART_DTYPE.itemsize
    g = abi.GPART_DTYPE.fields
    for off, name in {"off_x": "x", "off_a_grav": "a_grav", "off_potential": "potential",
                      "off_mass": "mass", "off_epsilon": "epsilon",
                      "off_time_bin": "time_bin"}.items():
        assert getattr(G, off) == g[name][1], (off, name)


def test_struct_part_offsets_match_survey():
    # offsets probed on the compiled reference
    f = abi.PART_DTYPE.fields
    expect = {"x": 16, "v": 40, "a_hydro": 52, "mass": 64, "h": 68, "u": 72, "u_dt": 76,
              "rho": 80, "div_v": 84, "laplace_u": 104, "wcount": 112, "f": 112,
              "time_bin": 137}
    for k, v in expect.items():
        assert f[k][1] == v, k
    g = abi.GPART_DTYPE.fields
    for k, v in {"x": 8, "v_full": 32, "a_grav": 44, "a_grav_mesh": 56, "potential": 68,
                 "mass": 76, "epsilon": 84, "time_bin": 88, "type": 89}.items():
        assert g[k][1] == v, k


def test_params_struct_size():
    # swh_hydro_params: 6 doubles + 4 floats + 2 ints + 8 floats + 2 ints + 3 doubles
    # + the dt_alpha_bins pointer (ABI v7)
    assert C.sizeof(abi.HydroParams) == 6 * 8 + 4 * 4 + 2 * 4 + 8 * 4 + 2 * 4 + 3 * 8 + 8
    assert abi.HydroParams.dt_alpha_bins.offset == 136
    # swh_grav_params: mesh scalars (40 B) + 2 floats + 4 ints of the MAC + r_cut_max
    assert C.sizeof(abi.GravParams) == 72
    assert abi.GravParams.r_cut_max.offset == 64
    # swh_gcell: start, count, split, progeny[8]; swh_grav_tree_stats: 5 int64
    assert C.sizeof(abi.GCell) == 96 == abi.GCELL_DTYPE.itemsize
    assert abi.GCell.loc.offset == 48 and abi.GCell.width.offset == 72
    assert C.sizeof(abi.GravTreeStats) == 72  # ABI v10: + int64 n_pp_truncated at 64
    assert abi.GravTreeStats.n_pp_truncated.offset == 64
    # swh_multipole: CoM, r_max, 35 terms, 5 powers, 2 floats
    assert C.sizeof(abi.Multipole) == 4 * 8 + 35 * 4 + 5 * 4 + 2 * 4


def test_aligned_parts():
    p = abi.new_parts(17)
    assert p.ctypes.data % 32 == 0
    q = abi.copy_parts(p)
    assert q.tobytes() == p.tobytes()
    assert np.all(q["time_bin"] == 0)


def test_adapter_layout_is_its_own_offsetof():
    """The adapter hands libswifthip the struct part / gpart layout it was
    compiled against (sizeof / offsetof in swh_swift_adapter.c), not the
    library's built-in default: here both see include/swift_compat.h, so they
    must agree field by field."""
    ad = lib.load_adapter()
    ad.swifthip_swift_part_layout.argtypes = [C.POINTER(abi.PartLayout)]
    ad.swifthip_swift_gpart_layout.argtypes = [C.POINTER(abi.GPartLayout)]
    mine, theirs = abi.PartLayout(), lib.part_layout()
    ad.swifthip_swift_part_layout(C.byref(mine))
    for name, _ in abi.PartLayout._fields_:
        assert getattr(mine, name) == getattr(theirs, name), name
    gm, gt = abi.GPartLayout(), lib.gpart_layout()
    ad.swifthip_swift_gpart_layout(C.byref(gm))
    for name, _ in abi.GPartLayout._fields_:
        assert getattr(gm, name) == getattr(gt, name), name
