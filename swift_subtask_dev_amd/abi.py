"""Python mirrors of the C ABI structures.

* ``PART_DTYPE`` / ``GPART_DTYPE``: numpy structured dtypes with the exact
  byte layout of SWIFT's default-configure ``struct part`` (SPHENIX, 160 B,
  src/hydro/SPHENIX/hydro_part.h:99-309) and ``struct gpart`` (multi-softening,
  96 B). The density/force union members overlap exactly as in C.
* ctypes mirrors of ``include/swifthip.h`` (params, cell views, layouts) and of
  the SWIFT field-name mirrors in ``include/swift_compat.h`` (cell, engine,
  runner, ...), used by the adapter and the oracle.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

# --------------------------------------------------------------------------
# struct part / struct gpart
# --------------------------------------------------------------------------
_PART_FIELDS = [
    ("id", "<i8", 0),
    ("gpart", "<u8", 8),
    ("x", ("<f8", (3,)), 16),
    ("v", ("<f4", (3,)), 40),
    ("a_hydro", ("<f4", (3,)), 52),
    ("mass", "<f4", 64),
    ("h", "<f4", 68),
    ("u", "<f4", 72),
    ("u_dt", "<f4", 76),
    ("rho", "<f4", 80),
    ("div_v", "<f4", 84),
    ("div_v_dt", "<f4", 88),
    ("div_v_previous_step", "<f4", 92),
    ("visc_alpha", "<f4", 96),
    ("v_sig", "<f4", 100),
    ("laplace_u", "<f4", 104),
    ("diff_alpha", "<f4", 108),
    # union member `density`
    ("wcount", "<f4", 112),
    ("wcount_dh", "<f4", 116),
    ("rho_dh", "<f4", 120),
    ("rot_v", ("<f4", (3,)), 124),
    # union member `force` (aliases the bytes above)
    ("f", "<f4", 112),
    ("pressure", "<f4", 116),
    ("soundspeed", "<f4", 120),
    ("h_dt", "<f4", 124),
    ("balsara", "<f4", 128),
    ("alpha_visc_max_ngb", "<f4", 132),
    ("rt_time_bin", "i1", 136),
    ("time_bin", "i1", 137),
    ("wakeup", "i1", 138),
    ("min_ngb_time_bin", "i1", 139),
    ("to_be_synchronized", "i1", 140),
]

PART_DTYPE = np.dtype(
    {
        "names": [f[0] for f in _PART_FIELDS],
        "formats": [f[1] for f in _PART_FIELDS],
        "offsets": [f[2] for f in _PART_FIELDS],
        "itemsize": 160,
    }
)

_GPART_FIELDS = [
    ("id_or_neg_offset", "<i8", 0),
    ("x", ("<f8", (3,)), 8),
    ("v_full", ("<f4", (3,)), 32),
    ("a_grav", ("<f4", (3,)), 44),
    ("a_grav_mesh", ("<f4", (3,)), 56),
    ("potential", "<f4", 68),
    ("potential_mesh", "<f4", 72),
    ("mass", "<f4", 76),
    ("old_a_grav_norm", "<f4", 80),
    ("epsilon", "<f4", 84),
    ("time_bin", "i1", 88),
    ("type", "i1", 89),
]
GPART_DTYPE = np.dtype(
    {
        "names": [f[0] for f in _GPART_FIELDS],
        "formats": [f[1] for f in _GPART_FIELDS],
        "offsets": [f[2] for f in _GPART_FIELDS],
        "itemsize": 96,
    }
)

# include/swift_compat.h struct xpart (SPHENIX): the drift's fields + padding
XPART_DTYPE = np.dtype(
    {
        "names": ["x_diff", "x_diff_sort", "v_full", "a_grav", "u_full"],
        "formats": [("<f4", 3), ("<f4", 3), ("<f4", 3), ("<f4", 3), "<f4"],
        "offsets": [0, 12, 24, 36, 48],
        "itemsize": 96,
    }
)

# include/swifthip.h SWH_ABI_VERSION: the ctypes layouts below are written for it
ABI_VERSION = 11

NUM_TIME_BINS = 56  # src/timeline.h:36
TIME_BIN_INHIBITED = NUM_TIME_BINS + 2
DEFAULT_LIST_SKIN = 0.01  # swifthip.h SWH_DEFAULT_LIST_SKIN (swh_tuning.list_skin)


def new_parts(n: int) -> np.ndarray:
    """Zeroed, 32-byte aligned struct part array (SWIFT_STRUCT_ALIGN)."""
    raw = np.zeros(n * 160 + 32, dtype=np.uint8)
    off = (-raw.ctypes.data) % 32
    return raw[off : off + n * 160].view(PART_DTYPE)


def new_xparts(n: int) -> np.ndarray:
    raw = np.zeros(n * 96 + 32, dtype=np.uint8)
    off = (-raw.ctypes.data) % 32
    return raw[off : off + n * 96].view(XPART_DTYPE)


def new_gparts(n: int) -> np.ndarray:
    raw = np.zeros(n * 96 + 32, dtype=np.uint8)
    off = (-raw.ctypes.data) % 32
    return raw[off : off + n * 96].view(GPART_DTYPE)


# --------------------------------------------------------------------------
# include/swifthip.h
# --------------------------------------------------------------------------
class PartLayout(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "stride", "off_id", "off_x", "off_v", "off_a_hydro", "off_mass", "off_h", "off_u",
        "off_u_dt", "off_rho", "off_div_v", "off_div_v_dt", "off_div_v_previous_step",
        "off_visc_alpha", "off_v_sig", "off_laplace_u", "off_diff_alpha", "off_wcount",
        "off_wcount_dh", "off_rho_dh", "off_rot_v", "off_f", "off_pressure",
        "off_soundspeed", "off_h_dt", "off_balsara", "off_alpha_visc_max_ngb",
        "off_time_bin", "off_min_ngb_time_bin", "off_gpart")]


class XPartLayout(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("stride", "off_v_full", "off_a_grav")]


class DriftParams(C.Structure):
    """swh_drift_params (== the oracle's oracle_drift_params)."""

    _fields_ = [("dt_drift", C.c_double), ("dt_kick_hydro", C.c_double),
                ("dt_kick_grav", C.c_double), ("dt_therm", C.c_double), ("min_u", C.c_float)]


class GPartLayout(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "stride", "off_x", "off_a_grav", "off_potential", "off_mass", "off_epsilon",
        "off_time_bin", "off_old_a_grav_norm")]


class HydroParams(C.Structure):
    """swh_hydro_params (identical layout to the oracle's oracle_params)."""

    _fields_ = [
        ("a", C.c_double), ("H", C.c_double), ("a2_inv", C.c_double),
        ("a_factor_sound_speed", C.c_double), ("a_factor_Balsara_eps", C.c_double),
        ("time_base", C.c_double),
        ("eta_neighbours", C.c_float), ("h_tolerance", C.c_float), ("h_max", C.c_float),
        ("h_min", C.c_float),
        ("max_smoothing_iterations", C.c_int32), ("use_mass_weighted_num_ngb", C.c_int32),
        ("visc_alpha", C.c_float), ("visc_alpha_max", C.c_float),
        ("visc_alpha_min", C.c_float), ("visc_length", C.c_float),
        ("diff_alpha", C.c_float), ("diff_beta", C.c_float), ("diff_alpha_max", C.c_float),
        ("diff_alpha_min", C.c_float),
        ("max_active_bin", C.c_int32), ("periodic", C.c_int32), ("dim", C.c_double * 3),
        ("dt_alpha_bins", C.POINTER(C.c_double)),
    ]

    def set_dt_alpha_bins(self, table) -> None:
        """Per-time-bin dt_alpha (cosmological runs, cosmo.dt_alpha_table);
        None restores the non-cosmological get_timestep. The array is kept
        alive by this object."""
        if table is None:
            self._dt_keep = None
            self.dt_alpha_bins = None
            return
        arr = (C.c_double * (NUM_TIME_BINS + 1))(*[float(v) for v in table])
        self._dt_keep = arr
        self.dt_alpha_bins = C.cast(arr, C.POINTER(C.c_double))


class GravParams(C.Structure):
    """swh_grav_params (identical layout to the oracle's oracle_grav_params):
    mesh scalars, then the M2P acceptance (gravity_props) fields."""

    _fields_ = [("periodic", C.c_int32), ("dim", C.c_float * 3), ("r_s_inv", C.c_float),
                ("r_cut_min", C.c_double), ("max_active_bin", C.c_int32),
                ("theta_crit", C.c_float), ("adaptive_tolerance", C.c_float),
                ("use_advanced_MAC", C.c_int32), ("use_gadget_tolerance", C.c_int32),
                ("use_tree_below_softening", C.c_int32),
                ("consider_truncation_in_MAC", C.c_int32), ("r_cut_max", C.c_double)]


class PMParams(C.Structure):
    """swh_pm_params (swh_gspace_pm_mesh)."""

    _fields_ = [("N", C.c_int32), ("off_a_grav_mesh", C.c_int32),
                ("off_potential_mesh", C.c_int32), ("reserved", C.c_int32),
                ("box_size", C.c_double), ("r_s", C.c_double), ("const_G", C.c_double)]


# struct gpart (multi-softening) offsets of the mesh fields (swift_compat.h)
GPART_OFF_A_GRAV_MESH = 56
GPART_OFF_POTENTIAL_MESH = 72


class GCell(C.Structure):
    """swh_gcell: a tree cell's gpart range, progeny and geometry."""

    _fields_ = [("start", C.c_int32), ("count", C.c_int32), ("split", C.c_int32),
                ("progeny", C.c_int32 * 8), ("reserved", C.c_int32),
                ("loc", C.c_double * 3), ("width", C.c_double * 3)]


GCELL_DTYPE = np.dtype({"names": ["start", "count", "split", "progeny", "loc", "width"],
                        "formats": ["<i4", "<i4", "<i4", ("<i4", 8), ("<f8", 3), ("<f8", 3)],
                        "offsets": [0, 4, 8, 12, 48, 72], "itemsize": 96})


class GravTreeStats(C.Structure):
    _fields_ = [("n_pp", C.c_int64), ("n_m2p", C.c_int64), ("n_m2l", C.c_int64),
                ("n_pp_tasks", C.c_int64), ("n_skipped", C.c_int64),
                ("ms_multipoles", C.c_float), ("ms_walk", C.c_float), ("ms_p2p", C.c_float),
                ("ms_m2p", C.c_float), ("ms_down", C.c_float), ("reserved", C.c_int32),
                ("n_pp_truncated", C.c_int64)]


MPOLE_TERMS = 35
# swh_multipole::M order (include/swifthip.h): struct multipole's member order
MPOLE_INDEX = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1),
               (2, 0, 0), (0, 2, 0), (0, 0, 2), (1, 1, 0), (1, 0, 1), (0, 1, 1),
               (3, 0, 0), (0, 3, 0), (0, 0, 3), (2, 1, 0), (2, 0, 1), (1, 2, 0), (0, 2, 1),
               (1, 0, 2), (0, 1, 2), (1, 1, 1),
               (4, 0, 0), (0, 4, 0), (0, 0, 4), (3, 1, 0), (3, 0, 1), (1, 3, 0), (0, 3, 1),
               (1, 0, 3), (0, 1, 3), (2, 2, 0), (2, 0, 2), (0, 2, 2), (2, 1, 1), (1, 2, 1),
               (1, 1, 2)]


class Multipole(C.Structure):
    """swh_multipole (== the oracle's oracle_multipole)."""

    _fields_ = [("CoM", C.c_double * 3), ("r_max", C.c_double), ("M", C.c_float * MPOLE_TERMS),
                ("power", C.c_float * 5), ("max_softening", C.c_float),
                ("min_old_a_grav_norm", C.c_float)]


class CellView(C.Structure):
    _fields_ = [("parts", C.c_void_p), ("count", C.c_int32), ("active", C.c_int32),
                ("loc", C.c_double * 3), ("width", C.c_double * 3)]


class GCellView(C.Structure):
    _fields_ = [("gparts", C.c_void_p), ("count", C.c_int32), ("active", C.c_int32),
                ("loc", C.c_double * 3), ("width", C.c_double * 3), ("CoM", C.c_double * 3),
                ("r_max", C.c_double), ("multipole", C.POINTER(Multipole))]


class SpaceInfo(C.Structure):
    """swh_space_info (include/swifthip.h)."""
    _fields_ = [("cdim", C.c_int32 * 3), ("ncell", C.c_int32), ("ngroups", C.c_int32),
                ("reserved", C.c_int32), ("cell_width", C.c_double * 3), ("h_max", C.c_double),
                ("loop_stats", C.c_int64 * 4), ("list_entries", C.c_int64),
                ("list_overflow", C.c_int32), ("list_valid", C.c_int32),
                ("dx_max", C.c_double), ("list_builds", C.c_int64)]


class Tuning(C.Structure):
    """swh_tuning (include/swifthip.h)."""
    _fields_ = [("cell_factor", C.c_int32), ("loop_variant", C.c_int32),
                ("group_size", C.c_int32), ("cell_scale", C.c_float), ("diag_mode", C.c_int32),
                ("list_capacity", C.c_int32), ("list_skin", C.c_float),
                ("list_keep", C.c_int32)]


class Leaf(C.Structure):
    _fields_ = [("start", C.c_int32), ("count", C.c_int32)]


LEAF_DTYPE = np.dtype([("start", "<i4"), ("count", "<i4")])
LEAF_PAIR_DTYPE = np.dtype([("j", "<i4"), ("truncated", "<i4"), ("allow_mpole", "<i4")])

FIELDS_DENSITY, FIELDS_GRADIENT, FIELDS_FORCE, FIELDS_DRIFT, FIELDS_ALL = 1, 2, 4, 8, 15
# halo record fields (swh_space_unpack_halo): h, rho, P + c, f + balsara, alphas
HALO_H, HALO_RHO, HALO_PC, HALO_F_BALSARA, HALO_ALPHAS, HALO_ALL = 1, 2, 4, 8, 16, 31
HALO_RECORD_FLOATS = 8


def default_hydro_params(dim=(1.0, 1.0, 1.0), periodic=True, **kw) -> HydroParams:
    """Non-cosmological engine scalars with SWIFT's defaults:
    hydro_props_init_no_hydro (src/hydro_properties.c:352-383) and the SPHENIX
    viscosity/diffusion defaults (src/hydro/SPHENIX/hydro_parameters.h)."""
    P = HydroParams()
    P.a = 1.0
    P.H = 0.0
    P.a2_inv = 1.0
    P.a_factor_sound_speed = 1.0
    P.a_factor_Balsara_eps = 1.0
    P.time_base = 0.0
    P.eta_neighbours = 1.2348
    P.h_tolerance = 1e-4
    P.h_max = np.finfo(np.float32).max
    P.h_min = 0.0
    P.max_smoothing_iterations = 30
    P.use_mass_weighted_num_ngb = 0
    P.visc_alpha, P.visc_alpha_max, P.visc_alpha_min, P.visc_length = 0.1, 2.0, 0.0, 0.05
    P.diff_alpha, P.diff_beta, P.diff_alpha_max, P.diff_alpha_min = 0.0, 1.0, 1.0, 0.0
    P.max_active_bin = NUM_TIME_BINS
    P.periodic = 1 if periodic else 0
    for k in range(3):
        P.dim[k] = dim[k]
    for k, v in kw.items():
        setattr(P, k, v)
    return P


# --------------------------------------------------------------------------
# include/swift_compat.h (SWIFT field-name mirrors)
# --------------------------------------------------------------------------
class Cosmology(C.Structure):
    _fields_ = [("a", C.c_double), ("H", C.c_double), ("a2_inv", C.c_double),
                ("a_factor_sound_speed", C.c_double), ("a_factor_Balsara_eps", C.c_double)]


class ViscosityGlobal(C.Structure):
    _fields_ = [("alpha", C.c_float), ("alpha_max", C.c_float), ("alpha_min", C.c_float),
                ("length", C.c_float)]


class DiffusionGlobal(C.Structure):
    _fields_ = [("alpha", C.c_float), ("beta", C.c_float), ("alpha_max", C.c_float),
                ("alpha_min", C.c_float)]


class HydroProps(C.Structure):
    _fields_ = [("eta_neighbours", C.c_float), ("h_tolerance", C.c_float),
                ("h_max", C.c_float), ("h_min", C.c_float),
                ("max_smoothing_iterations", C.c_int), ("use_mass_weighted_num_ngb", C.c_int),
                ("viscosity", ViscosityGlobal), ("diffusion", DiffusionGlobal)]


class Space(C.Structure):
    _fields_ = [("periodic", C.c_int), ("dim", C.c_double * 3),
                ("cells_top", C.c_void_p), ("cells_with_particles_top", C.POINTER(C.c_int)),
                ("nr_cells_with_particles", C.c_int)]


class PmMesh(C.Structure):
    _fields_ = [("periodic", C.c_int), ("dim", C.c_double * 3), ("r_s_inv", C.c_float),
                ("r_cut_min", C.c_double), ("r_cut_max", C.c_double)]


_TENSOR_NAMES = ["%d%d%d" % t for t in MPOLE_INDEX]


class GravTensor(C.Structure):
    """include/swift_compat.h struct grav_tensor (SWIFT multipole_struct.h:36)."""

    _fields_ = [("F_" + n, C.c_float) for n in _TENSOR_NAMES] + [("interacted", C.c_int)]


class MultipoleStruct(C.Structure):
    """include/swift_compat.h struct multipole (SWIFT multipole_struct.h:110):
    the dipole terms are not stored."""

    _fields_ = ([("vel", C.c_float * 3), ("max_delta_vel", C.c_float * 3),
                 ("min_delta_vel", C.c_float * 3), ("max_softening", C.c_float),
                 ("min_old_a_grav_norm", C.c_float), ("power", C.c_float * 5)] +
                [("M_" + n, C.c_float) for n in _TENSOR_NAMES if n not in ("100", "010", "001")])


class GravityTensors(C.Structure):
    _fields_ = [("pot", GravTensor), ("m_pole", MultipoleStruct), ("CoM", C.c_double * 3),
                ("CoM_rebuild", C.c_double * 3), ("r_max", C.c_double),
                ("r_max_rebuild", C.c_double)]

    def set_from(self, m: Multipole) -> None:
        """Fill from a swh_multipole (the adapter's inverse map)."""
        for k in range(3):
            self.CoM[k] = m.CoM[k]
        self.r_max = m.r_max
        mp = self.m_pole
        mp.max_softening = m.max_softening
        mp.min_old_a_grav_norm = m.min_old_a_grav_norm
        for k in range(5):
            mp.power[k] = m.power[k]
        for t, n in enumerate(_TENSOR_NAMES):
            if n not in ("100", "010", "001"):
                setattr(mp, "M_" + n, m.M[t])


class GravityProps(C.Structure):
    """include/swift_compat.h struct gravity_props (the MAC fields)."""

    _fields_ = [("use_advanced_MAC", C.c_int), ("use_adaptive_tolerance", C.c_int),
                ("use_gadget_tolerance", C.c_int), ("adaptive_tolerance", C.c_float),
                ("theta_crit", C.c_double), ("use_tree_below_softening", C.c_int),
                ("consider_truncation_in_MAC", C.c_int)]


class Engine(C.Structure):
    _fields_ = [("s", C.POINTER(Space)), ("cosmology", C.POINTER(Cosmology)),
                ("hydro_properties", C.POINTER(HydroProps)), ("mesh", C.POINTER(PmMesh)),
                ("gravity_properties", C.POINTER(GravityProps)),
                ("max_active_bin", C.c_int8), ("ti_current", C.c_longlong),
                ("time_base", C.c_double), ("policy", C.c_int), ("nodeID", C.c_int)]


class Runner(C.Structure):
    _fields_ = [("e", C.POINTER(Engine)), ("id", C.c_int)]


class CellHydro(C.Structure):
    _fields_ = [("parts", C.c_void_p), ("xparts", C.c_void_p), ("sort", C.c_void_p * 13),
                ("count", C.c_int), ("h_max", C.c_float), ("h_max_old", C.c_float),
                ("h_max_active", C.c_float), ("dx_max_part", C.c_float),
                ("dx_max_sort", C.c_float), ("dx_max_sort_old", C.c_float),
                ("dx_max_part_old", C.c_float),
                ("sorted", C.c_uint16), ("ti_end_min", C.c_longlong),
                ("ti_old_part", C.c_longlong)]


class CellGrav(C.Structure):
    _fields_ = [("parts", C.c_void_p), ("count", C.c_int),
                ("multipole", C.POINTER(GravityTensors)), ("ti_end_min", C.c_longlong),
                ("ti_old_part", C.c_longlong), ("ti_old_multipole", C.c_longlong)]


class Cell(C.Structure):
    _fields_ = [("loc", C.c_double * 3), ("width", C.c_double * 3), ("dmin", C.c_float),
                ("split", C.c_int), ("nodeID", C.c_int), ("progeny", C.c_void_p * 8),
                ("parent", C.c_void_p), ("hydro", CellHydro), ("grav", CellGrav)]


class EngineBundle:
    """Owns a compat engine + the structs it points to (keeps them alive)."""

    def __init__(self, dim=(1.0, 1.0, 1.0), periodic=True, ti_current=8, params=None,
                 max_active_bin=NUM_TIME_BINS, mesh=None, gravity_props=None):
        P = params or default_hydro_params(dim, periodic)
        self.params = P
        self.space = Space(1 if periodic else 0, (C.c_double * 3)(*dim))
        self.cosmo = Cosmology(P.a, P.H, P.a2_inv, P.a_factor_sound_speed,
                               P.a_factor_Balsara_eps)
        self.hp = HydroProps(P.eta_neighbours, P.h_tolerance, P.h_max, P.h_min,
                             P.max_smoothing_iterations, P.use_mass_weighted_num_ngb,
                             ViscosityGlobal(P.visc_alpha, P.visc_alpha_max, P.visc_alpha_min,
                                             P.visc_length),
                             DiffusionGlobal(P.diff_alpha, P.diff_beta, P.diff_alpha_max,
                                             P.diff_alpha_min))
        self.mesh = mesh or PmMesh(0, (C.c_double * 3)(*dim), 0.0, 0.0, 0.0)
        self.gprops = gravity_props or GravityProps(0, 0, 0, 0.0, 0.5, 0, 0)
        self.engine = Engine(C.pointer(self.space), C.pointer(self.cosmo), C.pointer(self.hp),
                             C.pointer(self.mesh), C.pointer(self.gprops), max_active_bin,
                             ti_current, P.time_base, 0, 0)
        self.runner = Runner(C.pointer(self.engine), 0)

    @property
    def runner_ptr(self):
        return C.byref(self.runner)


def copy_parts(p: np.ndarray) -> np.ndarray:
    """Byte-exact copy (numpy's structured copy leaves padding bytes
    uninitialised)."""
    out = new_parts(len(p)) if p.dtype == PART_DTYPE else new_gparts(len(p))
    out.view(np.uint8)[:] = np.ascontiguousarray(p).view(np.uint8)
    return out
