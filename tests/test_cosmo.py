"""CPU tests of the host-side cosmology (swift_subtask_dev_amd/cosmo.py): the
time integral behind cosmology_get_delta_time (src/cosmology.c:1287-1307)
against closed forms, the integer time line (src/timeline.h:59-114) and the
per-bin dt_alpha table of the extra ghost (src/runner_ghost.c:1038-1046)."""
from __future__ import annotations

import math

import numpy as np

from swift_subtask_dev_amd import abi, cosmo


def t_eds(a, H0=1.0):
    """Einstein-de Sitter: t(a) = 2 / (3 H0) a^(3/2)."""
    return 2.0 / (3.0 * H0) * a ** 1.5


def t_lcdm(a, Om, Ol, H0=1.0):
    """Flat LCDM: t(a) = 2 / (3 H0 sqrt(OL)) asinh(sqrt(OL / Om) a^(3/2))."""
    return 2.0 / (3.0 * H0 * math.sqrt(Ol)) * math.asinh(math.sqrt(Ol / Om) * a ** 1.5)


def test_time_line():
    assert cosmo.get_integer_timestep(0) == 0
    assert cosmo.get_integer_timestep(3) == 16
    # the reference subtracts one: the step that ENDS at ti_current
    assert cosmo.get_integer_time_begin(64, 3) == 48
    assert cosmo.get_integer_time_begin(65, 3) == 64
    assert cosmo.MAX_NR_TIMESTEPS == 1 << 57


def test_delta_time_eds_and_lcdm():
    for cm, tfun in ((cosmo.Cosmology(Omega_cdm=1.0, Omega_b=0.0, Omega_lambda=0.0,
                                      H0=2.5), lambda a: t_eds(a, 2.5)),
                     (cosmo.Cosmology(), lambda a: t_lcdm(a, 0.2587 + 0.0486, 0.6927))):
        ti_of = lambda a: int(round((math.log(a) - cm.log_a_begin) / cm.time_base))  # noqa
        for a0, a1 in ((0.05, 0.1), (0.3, 0.9), (0.5, 0.5001)):
            t0, t1 = ti_of(a0), ti_of(a1)
            exact = tfun(cm.scale_factor(t1)) - tfun(cm.scale_factor(t0))
            got = cm.get_delta_time(t0, t1)
            # linear interpolation on 30,000 log-a points (interp_table):
            # ~1e-8 on long intervals, the table slope on short ones
            tol = 1e-7 if a1 - a0 > 0.01 else 2e-4
            assert abs(got - exact) <= tol * exact, (a0, a1, got, exact)


def test_dt_alpha_table():
    cm = cosmo.Cosmology()
    ti = 1 << 40
    tab = cosmo.dt_alpha_table(cm, ti)
    assert tab.shape == (abi.NUM_TIME_BINS + 1,) and tab[0] == 0.0
    for b in (1, 5, 20, 38):
        step = 1 << (b + 1)
        begin = step * ((ti - 1) // step)
        assert tab[b] == cm.get_delta_time(begin, begin + step)
    # dt ~ (d t / d log a) * d log a for small bins: doubling per bin
    assert np.allclose(tab[11:21] / tab[10:20], 2.0, rtol=1e-3)


def test_cosmological_params():
    cm = cosmo.Cosmology()
    ti = 1 << 55
    P = cosmo.cosmological_params(cm, ti)
    a = cm.scale_factor(ti)
    assert P.a == a and abs(P.a2_inv * a * a - 1) < 1e-15
    assert abs(P.H - cm.H0 * math.sqrt(0.3073 / a ** 3 + 0.6927)) < 1e-12 * P.H
    assert abs(P.a_factor_sound_speed - a ** -1.0) < 1e-12  # a^(-3 (gamma-1) / 2)
    assert abs(P.a_factor_Balsara_eps - a ** -2.0) < 1e-12  # a^((1 - 3 gamma) / 2)
    tab = np.ctypeslib.as_array(P.dt_alpha_bins, shape=(abi.NUM_TIME_BINS + 1,))
    assert np.array_equal(tab, cosmo.dt_alpha_table(cm, ti))
    P.set_dt_alpha_bins(None)
    assert not P.dt_alpha_bins
