"""Scenario builders mirroring the reference's hot-path unit tests
(tests/test27cells.c, tests/test125cells.c, tests/testActivePair.c,
tests/testPeriodicBC.c), shared by the oracle tests and the GPU parity tests.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import oracle_lib as O
from swift_subtask_dev_amd import abi, ics

VEL = ["zero", "random", "divergent", "rotating"]


def concat_parts(chunks):
    n = sum(len(c) for c in chunks)
    out = abi.new_parts(n)
    bounds = []
    s = 0
    for c in chunks:
        out[s:s + len(c)] = c
        bounds.append((s, s + len(c)))
        s += len(c)
    return out, bounds


def cells_grid(ncell_side: int, n: int, size=1.0, h=1.23485, rho=1.0, pert=0.0,
               vel="zero", h_pert=0.0, seed=0, shuffle=True):
    """ncell_side^3 cells of n^3 particles each, cell (i,j,k) at offset
    (i,j,k)*size, ordered i*side^2 + j*side + k (test27cells.c:520-531)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    chunks, locs = [], []
    pid = 0
    for i in range(ncell_side):
        for j in range(ncell_side):
            for k in range(ncell_side):
                off = (i * size, j * size, k * size)
                c = ics.make_cell(n, off, size, h, rho, pid, pert, vel, h_pert, rng,
                                  shuffle=shuffle)
                pid += len(c)
                chunks.append(c)
                locs.append(off)
    parts, bounds = concat_parts(chunks)
    return parts, bounds, locs


def zero_density_fields(parts):
    for f in ("rho", "wcount", "wcount_dh", "rho_dh", "div_v", "laplace_u"):
        parts[f] = 0
    parts["rot_v"] = 0


def density_columns(sub: np.ndarray, end: bool = True) -> np.ndarray:
    """Columns of test27cells.c dump_particle_fields after end_calculation:
    ID, x, v, rho, rho_dh, wcount (neighbour number), wcount_dh, div_v, rot_v."""
    return np.column_stack([
        sub["id"].astype(np.float64), sub["x"], sub["v"], sub["rho"], sub["rho_dh"],
        sub["wcount"], sub["wcount_dh"], sub["div_v"], sub["rot_v"]])


def end_calculation(sub: np.ndarray, P, kernel="cubic-spline"):
    """test27cells.c end_calculation: hydro_end_density, then wcount *= h^3 *
    kernel_norm (via the oracle's restated hydro_end_density)."""
    f = O.fn("f32", "part_end_density", kernel)
    norm = O.load("f32", kernel).orf_kernel_norm()
    for i in range(len(sub)):
        f(sub[i:i + 1].ctypes.data, C.byref(P))
    h = sub["h"].astype(np.float32)
    sub["wcount"] = (sub["wcount"] * (h * h * h)) * np.float32(norm)


def run27(parts, bounds, locs, backend: str, P, engine=None, main=13, loops="density",
          subset=False, kernel="cubic-spline"):
    """Density loop of test27cells.c:566-582 on the main cell: 26 pairs +
    self. backend: 'sorted' (oracle restatement of DOPAIR1/DOSELF1), 'brute'
    (tools.c pairs_all_density/self_all_density), 'adapter' (GPU through the
    SWIFT-signature adapter; caller passes the adapter lib)."""
    eb = engine or abi.EngineBundle(dim=(3.0, 3.0, 3.0), periodic=True, params=P)
    cs = O.CellSet(parts, bounds, locs, 1.0)
    if backend in ("sorted", "adapter"):
        cs.sort_all()
    r = eb.runner_ptr
    ncell = len(bounds)
    if backend == "sorted":
        pair = O.fn("f32", "dopair1_branch", kernel)
        slf = O.fn("f32", "doself1_branch", kernel)
        for j in range(ncell):
            if j != main:
                assert pair(C.addressof(eb.runner), cs.ptr(main), cs.ptr(j), 0) == 0
        assert slf(C.addressof(eb.runner), cs.ptr(main), 0) == 0
    elif backend == "brute":
        pair = O.fn("f32", "pairs_all_density", kernel)
        slf = O.fn("f32", "self_all_density", kernel)
        for j in range(ncell):
            if j != main:
                pair(C.addressof(eb.runner), cs.ptr(main), cs.ptr(j))
        slf(C.addressof(eb.runner), cs.ptr(main))
    elif backend == "adapter":
        from swift_subtask_dev_amd import lib as L
        ad = L.load_adapter(kernel)
        ad.swifthip_swift_clear_error()
        if subset:
            s, e = bounds[main]
            ind = (C.c_int * (e - s))(*range(e - s))
            for j in range(ncell):
                if j != main:
                    ad.runner_dopair_subset_branch_density(C.addressof(eb.runner), cs.ptr(main),
                                                           cs.cells[main].hydro.parts, ind,
                                                           e - s, cs.ptr(j))
            ad.runner_doself_subset_branch_density(C.addressof(eb.runner), cs.ptr(main),
                                                   cs.cells[main].hydro.parts, ind, e - s)
        else:
            for j in range(ncell):
                if j != main:
                    ad.runner_dopair1_branch_density(C.addressof(eb.runner), cs.ptr(main),
                                                     cs.ptr(j))
            ad.runner_doself1_branch_density(C.addressof(eb.runner), cs.ptr(main))
        err = ad.swifthip_swift_last_error()
        assert not err, err
    cs.free_sorts()
    return cs
