"""Overlap of a batch phase with host work ("overlap with
the CPU runners"): the batch calls only enqueue on the space's stream, and
swh_space_query / swh_gspace_query tell a scheduler without waiting whether
the phase has finished -- the point where SWIFT's dependent task (the ghost
after the density loop: ghost_in / ghost_out, src/engine_maketasks.c:2313-2316)
becomes ready. Meanwhile the calling thread runs other work (here: the CPU
oracle's density loop of another box, as a runner would take another task).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
from swift_subtask_dev_amd import abi, ics

pytestmark = pytest.mark.gpu


def test_density_phase_overlaps_host_work(gpu_ctx):
    from swift_subtask_dev_amd import lib
    P = abi.default_hydro_params()
    parts = ics.sedov_box(48, velocity="divergent", seed=5)  # ~110k parts: a ms-scale phase
    sp = lib.HydroSpace(gpu_ctx)
    sp.upload(abi.copy_parts(parts))
    sp.rebuild(P)
    sp.sync()
    assert sp.done()  # nothing queued
    # reference: the same phase run synchronously
    sp.init_parts(P)
    n_ref = sp.density(P)
    ref = abi.copy_parts(parts)
    sp.download(ref, abi.FIELDS_DENSITY)

    # the phase as a task: enqueue, return at once
    sp.init_parts(P)
    sp.density(P, count=False)
    busy_seen = not sp.done()
    # host work while the GPU runs (another cell's density on the CPU oracle)
    other = ics.sedov_box(10, velocity="divergent", seed=6)
    O.fn("f32", "init_parts")(other.ctypes.data, len(other), C.byref(P))
    n_cpu = O.fn("f64", "box_density")(other.ctypes.data, len(other), C.byref(P), None)
    polls = 0
    while not sp.done():
        polls += 1
    got = abi.copy_parts(parts)
    sp.download(got, abi.FIELDS_DENSITY)
    assert busy_seen, "the density phase had finished before the first query"
    assert n_cpu > 0 and n_ref > 0
    for f in ("rho", "rho_dh", "wcount", "wcount_dh", "div_v", "rot_v"):
        assert np.array_equal(got[f], ref[f]), f
    sp.close()


def test_gspace_query(gpu_ctx):
    from swift_subtask_dev_amd import lib
    gs = lib.GravSpace(gpu_ctx)
    assert gs.done()
    gs.sync()
    assert gs.done()
    gs.close()
