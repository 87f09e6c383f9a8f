"""The boundary's threading contract (SURVEY 8b "Threading"): SWIFT calls the
hydro task entries concurrently from nr_threads runner pthreads, each task
holding cell_locktree on its cells (src/task.c:866-868 self, 1031-1037 pair),
so concurrent tasks touch disjoint particles. The adapter leases one HIP
stream + staging buffers per calling thread (include/swifthip.h "Context").

The test drives the SWIFT-signature entries from 8 Python threads at once
(ctypes releases the GIL for the foreign call) on a 4x4x4 periodic grid of
cells, in three phases separated by barriers -- every self task, then the
x-pairs (2k, 2k+1), then the x-pairs (2k+1, 2k+2) -- so no two concurrent
tasks share a cell, exactly what cell locks guarantee. Every cell then sees
the same sequence of tasks as in a serial run, and the results must be
bitwise equal to the serial run's, for the density and the force loop.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np
import pytest

import oracle_lib as O
import scenarios as S
from swift_subtask_dev_amd import abi

pytestmark = pytest.mark.gpu

SIDE = 4
NTHREADS = 8


def _grid(seed):
    parts, bounds, locs = S.cells_grid(SIDE, 5, vel="divergent", h_pert=1.2, pert=0.1, seed=seed)
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
    return parts, bounds, locs


def _cid(i, j, k):
    return (i % SIDE) * SIDE * SIDE + (j % SIDE) * SIDE + (k % SIDE)


def _phases():
    selfs = [("self", c) for c in range(SIDE ** 3)]
    even = [("pair", _cid(i, j, k), _cid(i + 1, j, k))
            for i in range(0, SIDE, 2) for j in range(SIDE) for k in range(SIDE)]
    odd = [("pair", _cid(i, j, k), _cid(i + 1, j, k))
           for i in range(1, SIDE, 2) for j in range(SIDE) for k in range(SIDE)]
    return [selfs, even, odd]


def _run(ad, eb, cs, loop, nthreads):
    self_fn = ad.runner_doself1_branch_density if loop == "density" else \
        ad.runner_doself2_branch_force
    pair_fn = ad.runner_dopair1_branch_density if loop == "density" else \
        ad.runner_dopair2_branch_force
    r = C.addressof(eb.runner)
    errors = []

    def work(tasks):
        for t in tasks:
            if t[0] == "self":
                self_fn(r, cs.ptr(t[1]))
            else:
                pair_fn(r, cs.ptr(t[1]), cs.ptr(t[2]))
        e = ad.swifthip_swift_last_error()  # thread-local error text
        if e:
            errors.append(e)

    for phase in _phases():
        if nthreads == 1:
            work(phase)
            continue
        chunks = [phase[k::nthreads] for k in range(nthreads)]
        ths = [threading.Thread(target=work, args=(c,)) for c in chunks]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    assert not errors, errors


@pytest.mark.parametrize("loop", ["density", "force"])
def test_concurrent_tasks_bitwise_equal_serial(loop):
    from swift_subtask_dev_amd import lib
    ad = lib.load_adapter()
    assert ad.swifthip_swift_init(0, 0) == 0
    side = float(SIDE)
    P = abi.default_hydro_params((side, side, side), True)
    out = []
    for nthreads in (1, NTHREADS, NTHREADS):
        parts, bounds, locs = _grid(seed=17)
        if loop == "density":
            S.zero_density_fields(parts)
        else:
            parts["a_hydro"] = 0
            parts["u_dt"] = 0
            parts["h_dt"] = 0
            parts["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
        eb = abi.EngineBundle(dim=(side, side, side), periodic=True, params=P)
        cs = O.CellSet(parts, bounds, locs, 1.0)
        cs.sort_all()
        ad.swifthip_swift_clear_error()
        _run(ad, eb, cs, loop, nthreads)
        cs.free_sorts()
        out.append(parts)
    fields = (("rho", "rho_dh", "wcount", "wcount_dh", "div_v", "rot_v") if loop == "density"
              else ("a_hydro", "u_dt", "h_dt", "min_ngb_time_bin"))
    for f in fields:
        assert np.abs(out[0][f]).max() > 0, f
        for k in (1, 2):
            np.testing.assert_array_equal(out[k][f], out[0][f], err_msg=f"{f} run {k}")
