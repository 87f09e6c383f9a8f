"""north_star's "stated tolerance" against the reference's own precision.

The reference runner keeps struct part in float and computes in float
(SURVEY.md §8 conventions; hydro_iact.h, runner_ghost.c). The GPU computes in
fp64. Its distance from the float restatement (liboracle_f32, the reference's
operation order) is therefore the float's own rounding, amplified where sums
cancel, plus the ghost's stop decision: runner_do_ghost stops a particle
once |h_new - h_old| <= eps h_old (eps = h_tolerance = 1e-4,
runner_ghost.c:1103, 1352), so a float and a double iteration can stop one
Newton step apart, up to h_tolerance.

Per field: the largest relative difference over all particles and its 99.9th
percentile (relative to max(|float value|, 1e-4 x the column maximum), the
floor of tolerance_125_*.dat's absolute limits). Measured (CPU, this
container, f64 oracle chain vs f32 oracle chain from the same unconverged
input; the GPU is held to these bars AND to "no farther from the float chain
than the f64 oracle is"):

  sedov128  h 1.00e-4 / 2.9e-7   rho 1.4e-5 / 7.1e-7   a_hydro 9.9e-4 / 2e-12
  eagle     h 1.00e-4 / 3.0e-7   rho 1.9e-4 / 6.8e-7   a_hydro 2.9e-2 / 4.1e-4
            u_dt 1.8e-2 / 1.1e-4   h_dt 1.3e-2 / 3.7e-4

  flow64    h 1.00e-4 / 2.9e-7   rho 3.2e-5 / 6.9e-7   a_hydro 4.8e-2 / 1.4e-3
            u_dt 5.1e-3 / 1.9e-4   h_dt 1.3e-3 / 2.7e-4   v_sig 2.6e-7 / 2.0e-7

The EAGLE stand-in's clumps have pressure-gradient forces that cancel to a
few per cent of the terms summed, so the float's rounding reaches ~3% of
a_hydro on the worst particles; the 99.9th percentile stays at 4e-4.

flow64 (round 6) is ics.flow_box(64): a converging, shearing flow with a
lumpy u, h off target and earlier switch state, so the artificial viscosity
of approaching pairs (mu_ij < 0), the diffusion and the switch evolution --
the terms the Sedov headline (v = 0) leaves at zero -- enter every field;
the viscous and pressure accelerations of neighbouring particles cancel, so
the float's a_hydro error reaches ~5% of the floor-limited value on the
worst particle (99.9th percentile 1.4e-3).

Interaction counts: the float and double pair criteria (r2 < H^2) differ only
on pairs within rounding of the kernel edge: |N_gpu - N_f32| <= 1e-6 N.
"""
from __future__ import annotations

import numpy as np

FLOOR = 1e-4  # x the column maximum of the float chain's values

# field -> (max relative difference, 99.9th percentile)
BARS = {
    "sedov128": {
        "h": (2e-4, 1e-6),
        "rho": (5e-5, 2e-6),
        "a_hydro": (2e-3, 1e-5),
        "u_dt": (1e-3, 1e-5),
        "h_dt": (1e-3, 1e-5),
    },
    "flow64": {
        "h": (2e-4, 1e-6),
        "rho": (1e-4, 2e-6),
        "a_hydro": (1e-1, 3e-3),
        "u_dt": (1e-2, 4e-4),
        "h_dt": (3e-3, 6e-4),
        "v_sig": (1e-6, 1e-6),
    },
    "eagle": {
        "h": (2e-4, 1e-6),
        "rho": (5e-4, 2e-6),
        "a_hydro": (6e-2, 1e-3),
        "u_dt": (4e-2, 3e-4),
        "h_dt": (3e-2, 1e-3),
    },
}
COUNT_REL = 1e-6


def rel_errors(a, b, floor=FLOOR):
    """Per-particle largest relative difference of a against b (vectors: the
    largest component), relative to max(|b|, floor x max |b|)."""
    x = np.asarray(a, dtype=np.float64).reshape(len(a), -1)
    y = np.asarray(b, dtype=np.float64).reshape(len(b), -1)
    fl = floor * max(float(np.abs(y).max()), 1e-300)
    return (np.abs(x - y) / np.maximum(np.abs(y), fl)).max(axis=1)


def summary(a, b, fields):
    """field -> (max, 99.9th percentile) of rel_errors."""
    out = {}
    for f in fields:
        e = rel_errors(a[f], b[f])
        out[f] = (float(e.max()), float(np.quantile(e, 0.999)))
    return out
