"""Host-side cosmology needed by the batch hydro path: the engine scalars a
cosmological step passes to the loops (swh_hydro_params) and the per-time-bin
dt_alpha of the extra ghost.

SWIFT's extra ghost evaluates, with cosmology, the physical duration of the
particle's current step (src/runner_ghost.c:1038-1046):

    ti_step  = get_integer_timestep(time_bin)                 timeline.h:59-63
    ti_begin = get_integer_time_begin(ti_current - 1, bin)    timeline.h:107-114
    dt_alpha = cosmology_get_delta_time(cosmo, ti_begin, ti_begin + ti_step)

dt_alpha depends only on (ti_current, time_bin), so the engine tabulates it
once per step for the 57 bins and hands the table to swh_extra_ghost
(swh_hydro_params.dt_alpha_bins); the device reads its bin's entry.

cosmology_get_delta_time (src/cosmology.c:1287-1307) interpolates
time_interp_table, the integral of dt = da / (a H(a)) from a_begin, on
cosmology_table_length = 30000 points uniform in log a (cosmology.c:46,
636-720; GSL's adaptive Gauss-Kronrod to 1e-10 relative there, a fixed
8-point Gauss-Legendre rule per table interval here: the same integral to
~1e-15), with E(a) of cosmology.c:185-195 (radiation, matter, curvature, and
dark energy w(a) = w_0 + w_a (1 - a), no massive neutrinos) and the linear
interpolation interp_table (cosmology.c:64-82). The scale-factor powers are
cosmology_update's (cosmology.c:225-270) for gamma = 5/3.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import abi

TABLE_LENGTH = 30000                       # cosmology.c:46
NUM_TIME_BINS = abi.NUM_TIME_BINS          # timeline.h:36
MAX_NR_TIMESTEPS = 1 << (NUM_TIME_BINS + 1)  # timeline.h:39
HYDRO_GAMMA = 5.0 / 3.0


def get_integer_timestep(bin_: int) -> int:
    """timeline.h:59-63."""
    return 0 if bin_ <= 0 else 1 << (bin_ + 1)


def get_integer_time_begin(ti_current: int, bin_: int) -> int:
    """timeline.h:107-114 (the reference subtracts one from its argument)."""
    dti = get_integer_timestep(bin_)
    return 0 if dti == 0 else dti * ((ti_current - 1) // dti)


@dataclass
class Cosmology:
    """The struct cosmology fields the hydro path reads (cosmology.c)."""

    Omega_cdm: float = 0.2587
    Omega_b: float = 0.0486
    Omega_lambda: float = 0.6927
    Omega_r: float = 0.0
    Omega_k: float = 0.0
    w_0: float = -1.0
    w_a: float = 0.0
    H0: float = 1.0
    a_begin: float = 1.0 / 51.0
    a_end: float = 1.0
    _table: np.ndarray = field(default=None, repr=False)

    @property
    def log_a_begin(self) -> float:
        return math.log(self.a_begin)

    @property
    def log_a_end(self) -> float:
        return math.log(self.a_end)

    @property
    def time_base(self) -> float:
        """cosmology.c:914: log a per integer time-line tick."""
        return (self.log_a_end - self.log_a_begin) / MAX_NR_TIMESTEPS

    def E(self, a):
        """cosmology.c:185-195 (w_tilde of :166-171)."""
        a = np.asarray(a, dtype=np.float64)
        a_inv = 1.0 / a
        w_tilde = (a - 1.0) * self.w_a - (1.0 + self.w_0 + self.w_a) * np.log(a)
        Om = self.Omega_cdm + self.Omega_b
        return np.sqrt(self.Omega_r * a_inv ** 4 + Om * a_inv ** 3 + self.Omega_k * a_inv ** 2
                       + self.Omega_lambda * np.exp(3.0 * w_tilde))

    def H(self, a):
        return self.H0 * self.E(a)

    # -- time_interp_table (cosmology.c:636-720) ------------------------------
    def time_table(self) -> np.ndarray:
        if self._table is None:
            n = TABLE_LENGTH
            dl = (self.log_a_end - self.log_a_begin) / n
            # t(a) = int da / (a H) = int dlog(a) / H; 8-point Gauss-Legendre
            # on every table interval [log a_begin + i dl, + (i+1) dl]
            xg, wg = np.polynomial.legendre.leggauss(8)
            lo = self.log_a_begin + dl * np.arange(n)
            nodes = lo[:, None] + 0.5 * dl * (xg[None, :] + 1.0)
            piece = (0.5 * dl * wg[None, :] / self.H(np.exp(nodes))).sum(axis=1)
            self._table = np.cumsum(piece)  # table[i] = int_{a_begin}^{a_table[i]}
        return self._table

    def _interp(self, x: float) -> float:
        """interp_table (cosmology.c:64-82)."""
        t = self.time_table()
        xx = (x - self.log_a_begin) / (self.log_a_end - self.log_a_begin) * TABLE_LENGTH
        i = int(xx)
        ii = min(TABLE_LENGTH - 1, i)
        if ii < 1:
            return t[0] * xx
        return t[ii - 1] + (t[ii] - t[ii - 1]) * (xx - ii)

    def get_delta_time(self, ti_start: int, ti_end: int) -> float:
        """cosmology_get_delta_time (cosmology.c:1287-1307)."""
        t1 = self._interp(self.log_a_begin + ti_start * self.time_base)
        t2 = self._interp(self.log_a_begin + ti_end * self.time_base)
        return t2 - t1

    def scale_factor(self, ti_current: int) -> float:
        """cosmology_update (cosmology.c:232)."""
        return self.a_begin * math.exp(ti_current * self.time_base)


def dt_alpha_table(cosmo: Cosmology, ti_current: int) -> np.ndarray:
    """dt_alpha of every time bin at ti_current (runner_ghost.c:1038-1046)."""
    out = np.zeros(NUM_TIME_BINS + 1, dtype=np.float64)
    for b in range(NUM_TIME_BINS + 1):
        ti_step = get_integer_timestep(b)
        if ti_step == 0:
            continue
        ti_begin = get_integer_time_begin(ti_current, b)
        out[b] = cosmo.get_delta_time(ti_begin, ti_begin + ti_step)
    return out


def cosmological_params(cosmo: Cosmology, ti_current: int, dim=(1.0, 1.0, 1.0),
                        periodic=True, **kw) -> abi.HydroParams:
    """swh_hydro_params of a cosmological step: a, H, a^-2 and the gamma = 5/3
    scale-factor powers of cosmology_update (cosmology.c:225-270), and the
    extra ghost's dt_alpha table."""
    a = cosmo.scale_factor(ti_current)
    P = abi.default_hydro_params(dim, periodic, **kw)
    P.a = a
    P.H = float(cosmo.H(a))
    P.a2_inv = 1.0 / (a * a)
    P.a_factor_sound_speed = a ** (-1.5 * (HYDRO_GAMMA - 1.0))
    P.a_factor_Balsara_eps = a ** (0.5 * (1.0 - 3.0 * HYDRO_GAMMA))
    P.time_base = cosmo.time_base
    P.set_dt_alpha_bins(dt_alpha_table(cosmo, ti_current))
    return P


# BASELINE config 5: the SmallCosmoVolume run's first step (small_cosmo_volume.yml)
SCV_FIRST_BIN = 47          # dt_max = 1e-2 in log a -> 2^48 ticks of time_base: bin 47
SCV_TI_CURRENT = 1 << 48    # the end of that first step (every bin <= 47 ends here)


def small_cosmo_volume_params(max_active_bin: int = SCV_FIRST_BIN) -> tuple:
    """(Cosmology, swh_hydro_params) of the SmallCosmoVolume stand-in's first
    step (ics.small_cosmo_volume): WMAP9 (Omega_cdm 0.2305, Omega_b 0.0455,
    Omega_lambda 0.724), H0 = 1e4 km/s per box length (70.3 km/s/Mpc x
    142.248 Mpc), a_begin = 1/51, a_end = 1; dt_max = 1e-2 in log a is
    2^48 ticks (time_base = ln(51) / 2^57), i.e. time bin 47, and the step
    ends at ti_current = 2^48 (a = 0.01976)."""
    from . import ics
    cm = Cosmology(Omega_cdm=ics.SCV_OMEGA_CDM, Omega_b=ics.SCV_OMEGA_B,
                   Omega_lambda=ics.SCV_OMEGA_L, H0=ics.SCV_H0, a_begin=ics.SCV_A_BEGIN, a_end=1.0)
    P = cosmological_params(cm, SCV_TI_CURRENT, max_active_bin=max_active_bin)
    return cm, P
