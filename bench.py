#!/usr/bin/env python
"""bench.py — directed particle-pair interactions/s (density + force loops)
on a SedovBlast_3D-like 128^3 box, MI355X, fp64, 1..N GPUs.

One step = one density loop + one force loop over every active particle of
the (per-GPU) 128^3 sub-volume — the two loops the metric names (SURVEY 8d:
"density + force; gradient reported separately"). Inputs are resident in HBM
before the timed region: a full SPHENIX chain (density, ghost h-iteration,
gradient, extra ghost, force) prepares converged smoothing lengths and the
force-loop inputs in an untimed setup. Timed per step, on the library's HIP
stream: hydro_init_part + density gather, hydro_reset_acceleration + force
gather.

Multi-GPU (default --scaling strong): the one 128^3 box is split into N
blocks (2x1x1, 2x2x1, 2x2x2); each rank holds its block + a read-only halo
(everything within gamma h_max), runs the loops for its own particles, and
between density and force refreshes the halo's rho point-to-point
(batch_isend_irecv over RCCL; swift_subtask_dev_amd/decomp.py). The timed step
includes that exchange. --scaling weak: N unit cubes along x, one x-slab per
rank, no exchange.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun ... bench.py --gpus N   (one process per GPU)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from swift_subtask_dev_amd import decomp  # noqa: E402  (numpy only)

METRIC = "particle-pair interactions/s (density+force) on SedovBlast_3D 128³; 1/2/4/8 GPU"
METRIC_EAGLE = "particle-pair interactions/s (density+force) on an EAGLE_6 stand-in (clustered)"
HBM_PEAK = 8.0e12       # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK = 78.6e12     # MI355X fp64 vector
S_IN_DENSITY, S_OUT_DENSITY = 45, 32   # SURVEY 8d algorithmic bytes per particle
S_IN_FORCE, S_OUT_FORCE = 77, 21
KERNEL_GAMMA = 1.825742  # H/h of the cubic spline (kernel_hydro.h:52): libswifthip.so's kernel
FLOPS_DENSITY, FLOPS_FORCE = 65, 146   # SURVEY 8d flops per directed interaction


RED_DEVICE = "cuda"  # device of the max/sum-over-ranks tensors
RANKS = {}  # world size, backend and the device of every rank (main)


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def cpu_share_threads():
    """This job's CPU share: OMP_NUM_THREADS (16 per GPU on the pool's boxes)
    or the CPUs it may run on, at most 16."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def run_cpu_worker(kind, arrays, meta, threads):
    """Run a CPU-baseline leg in a child process that never imports torch, so
    its OpenMP runtime starts with one thread per physical core of this job's
    share, pinned (OMP_PLACES=cores, OMP_PROC_BIND=close) -- torch's libgomp
    is the one the oracle binds to and reads its environment once, at torch's
    import. Inputs travel through an .npz under /tmp."""
    import subprocess
    import tempfile

    with tempfile.TemporaryDirectory(prefix="swh_cpu_") as d:
        path = os.path.join(d, "in.npz")
        np.savez(path, **arrays)
        env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PLACES="cores",
                   OMP_PROC_BIND="close")
        cmd = [sys.executable, str(Path(__file__).resolve()), "--cpu-worker", kind,
               "--cpu-input", path, "--cpu-meta", json.dumps(meta)]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            raise RuntimeError(f"cpu worker failed ({r.returncode}): {r.stderr[-2000:]}")
        return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def cpu_worker_main(kind, path, meta):
    """The child of run_cpu_worker: the oracle's float restatement timed on
    this process's pinned threads (test infrastructure: bench's cpu_baseline
    leg only)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    from swift_subtask_dev_amd import abi

    z = np.load(path)
    threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    out = {"threads": threads}
    if kind == "hydro":
        parts = z["parts"].view(abi.PART_DTYPE).reshape(-1)
        P = abi.default_hydro_params(tuple(meta["dim"]), True)
        P.max_active_bin = meta["max_active_bin"]
        eb = abi.EngineBundle(dim=tuple(P.dim), periodic=True, params=P,
                              max_active_bin=P.max_active_bin)
        new, run, free = (O.fn("f32", n) for n in ("cellgrid_new", "cellgrid_run",
                                                    "cellgrid_free"))
        # separate copies: the density/force union must keep the force inputs
        gd = new(parts.ctypes.data, len(parts), float(P.dim[0]), meta["cdim"])
        gf = new(parts.ctypes.data, len(parts), float(P.dim[0]), meta["cdim"])
        try:
            times = []
            for r in range(meta["runs"] + 1):  # first run = warm-up
                td = run(gd, C.addressof(eb.runner), 0, threads)
                tf = run(gf, C.addressof(eb.runner), 2, threads)
                if r > 0:
                    times.append(td + tf)
            out["seconds_share"] = statistics.median(times)
            # one pinned thread: the per-core rate (one run, memory already warm)
            out["seconds_1"] = (run(gd, C.addressof(eb.runner), 0, 1) +
                                run(gf, C.addressof(eb.runner), 2, 1))
        finally:
            free(gd)
            free(gf)
    elif kind == "hydro_tree":
        # SWIFT's cell tree + DOSUB recursion (clustered inputs)
        parts = z["parts"].view(abi.PART_DTYPE).reshape(-1)
        P = abi.default_hydro_params(tuple(meta["dim"]), True)
        P.max_active_bin = meta["max_active_bin"]
        eb = abi.EngineBundle(dim=tuple(P.dim), periodic=True, params=P,
                              max_active_bin=P.max_active_bin)
        new, run, free, ncells = (O.fn("f32", n) for n in ("celltree_new", "celltree_run",
                                                            "celltree_free", "celltree_ncells"))
        td0 = time.perf_counter()
        gd = new(parts.ctypes.data, len(parts), float(P.dim[0]), meta["cdim"], meta["splitsize"])
        gf = new(parts.ctypes.data, len(parts), float(P.dim[0]), meta["cdim"], meta["splitsize"])
        out["seconds_tree_build"] = (time.perf_counter() - td0) / 2
        out["cells"] = int(ncells(gd))
        try:
            times = []
            for r in range(meta["runs"] + 1):  # first run = warm-up
                td = run(gd, C.addressof(eb.runner), 0, threads)
                tf = run(gf, C.addressof(eb.runner), 2, threads)
                if r > 0:
                    times.append(td + tf)
            out["seconds_share"] = statistics.median(times)
        finally:
            free(gd)
            free(gf)
    elif kind == "grav":
        G = abi.GravParams.from_buffer_copy(z["G"].tobytes())
        g = z["gparts"].view(abi.GPART_DTYPE).reshape(-1).copy()
        leaves, offs, pairs = z["leaves"], z["offs"], z["pairs"]
        f = O.fn("f32", "grav_pp_leaves")
        times, n = [], 0
        for r in range(meta["runs"] + 1):
            t0 = time.perf_counter()
            n = f(g.ctypes.data, leaves.ctypes.data, len(leaves), offs.ctypes.data,
                  pairs.ctypes.data, C.byref(G), None, None)
            if r > 0:
                times.append(time.perf_counter() - t0)
        out["seconds_share"] = statistics.median(times)
        out["interactions"] = int(n)
    elif kind == "cosmo":
        from swift_subtask_dev_amd import cosmo
        parts = z["parts"].view(abi.PART_DTYPE).reshape(-1)
        _, P = cosmo.small_cosmo_volume_params()  # the GPU step's engine scalars
        eb = abi.EngineBundle(dim=(1.0, 1.0, 1.0), periodic=True, params=P,
                              max_active_bin=int(P.max_active_bin))
        new, run, free = (O.fn("f32", n) for n in ("cellgrid_new", "cellgrid_run",
                                                    "cellgrid_free"))
        gd = new(parts.ctypes.data, len(parts), 1.0, meta["cdim"])
        gf = new(parts.ctypes.data, len(parts), 1.0, meta["cdim"])
        try:
            run(gd, C.addressof(eb.runner), 0, threads)  # warm-up
            th = run(gd, C.addressof(eb.runner), 0, threads) + run(gf, C.addressof(eb.runner),
                                                                    2, threads)
        finally:
            free(gd)
            free(gf)
        G = abi.GravParams.from_buffer_copy(z["G"].tobytes())
        g = z["gparts"].view(abi.GPART_DTYPE).reshape(-1).copy()
        cells, tops, pc = z["cells"].view(abi.GCELL_DTYPE), z["tops"], z["pairs"]
        stats = (C.c_longlong * 6)()
        t0 = time.perf_counter()
        O.fn("f32", "grav_tree")(g.ctypes.data, len(g), cells.ctypes.data, len(cells),
                                 tops.ctypes.data, len(tops), pc.ctypes.data, len(pc) // 2,
                                 C.byref(G), stats, None)
        out["seconds_gravity"] = time.perf_counter() - t0
        out["seconds_hydro"] = th
        out["seconds_share"] = th + out["seconds_gravity"]
        out["tree_stats"] = list(stats)
    print(json.dumps(out), flush=True)


def cgroup_cpu_quota():
    """The CPU bandwidth limit of this job's cgroup (v2 cpu.max, or v1
    cfs_quota_us / cfs_period_us): CPUs' worth of time, or None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_baseline(parts, P, n_density, n_force, runs=3, threads=None):
    """The oracle's float restatement of DOSELF1/DOPAIR1 + DOSELF2/DOPAIR2
    (sorted pseudo-Verlet loops) over a cdim=20 periodic cell grid (kind
    "port"; the reference's own build is unavailable), timed on pinned
    threads, one per physical core (OMP_PLACES=cores):

      * `value`: this job's CPU share (16 threads per GPU on the pool's boxes),
        median of `runs` after a warm-up, and one pinned thread;
      * `full_host`: as many pinned threads as the host has physical cores and
        the job's cgroup CPU quota allows (both recorded), measured -- the
        north_star's "host cores of the same box";
      * `calibration`: the port runs at 0.72x the reference build's rate on
        one thread and 1.09x on eight (profiles/cpu_calibration.json, SURVEY 6
        recipe in the build container), so `reference_equivalent` divides
        the port's rates by the factor of its thread regime."""
    threads = threads or cpu_share_threads()
    w = run_cpu_worker("hydro", {"parts": np.ascontiguousarray(parts).view(np.uint8)},
                       {"dim": list(P.dim), "max_active_bin": int(P.max_active_bin),
                        "cdim": 20, "runs": runs}, threads)
    t, t1 = w["seconds_share"], w["seconds_1"]
    n = n_density + n_force
    host = host_cpu_info()
    phys = host.get("physical_cores") or threads
    quota = cgroup_cpu_quota()
    host["cgroup_cpu_quota"] = quota
    eff = (n / t / threads) / (n / t1)  # per-thread efficiency of the share run
    calib = None
    cpath = ROOT / "profiles" / "cpu_calibration.json"
    if cpath.exists():
        calib = json.loads(cpath.read_text())
    f1 = f8 = None
    if calib:
        f1 = calib["threads"]["1"]["port_over_reference"]
        f8 = calib["threads"]["8"]["port_over_reference"]
    out = {
        "value": n / t,
        "unit": "interactions/s",
        "cores": threads,
        "kind": "port",
        "pinning": "one thread per physical core (OMP_PLACES=cores, OMP_PROC_BIND=close), "
                   "child process without torch",
        "host": host,
        "calibration": calib,
        "sample": f"full 128^3 box, density+force loops (float restatement of DOSELF1/DOPAIR1/"
                  f"DOSELF2/DOPAIR2, cdim=20 cells), median of {runs} runs after 1 warm-up on "
                  f"{threads} pinned threads ({t:.3f} s per step); one pinned thread "
                  f"{t1:.3f} s per step",
        "seconds_per_step": t,
        "single_core": {"value": n / t1, "seconds_per_step": t1},
        "reference_equivalent": ({"value": n / t / f8, "single_core": n / t1 / f1,
                                  "basis": f"port rates / {f8:.3f} (multi-thread) and / "
                                           f"{f1:.3f} (one thread): the reference build's rate "
                                           "on the calibration recipe"} if calib else None),
        "full_host_projected": {
            "value": n / t1 * phys * eff, "cores": phys,
            "basis": f"one-thread rate x {phys} physical cores x the {eff:.3f} per-thread "
                     f"efficiency of the {threads}-thread run"},
    }
    # every physical core the job may use, measured
    allowed = phys if quota is None else min(phys, max(1, int(quota)))
    try:
        aff = len(os.sched_getaffinity(0))
        allowed = min(allowed, aff)
    except AttributeError:
        pass
    if allowed > threads:
        try:
            wf = run_cpu_worker("hydro", {"parts": np.ascontiguousarray(parts).view(np.uint8)},
                                {"dim": list(P.dim), "max_active_bin": int(P.max_active_bin),
                                 "cdim": 20, "runs": 1}, allowed)
            out["full_host"] = {"value": n / wf["seconds_share"], "cores": allowed,
                                "seconds_per_step": wf["seconds_share"],
                                "limit": f"min({phys} physical cores, cgroup quota {quota}, "
                                         f"affinity)",
                                "sample": "the same box and loops, 1 run after 1 warm-up"}
            if calib:
                out["full_host"]["reference_equivalent"] = n / wf["seconds_share"] / f8
        except Exception as e:  # report, never fake
            out["full_host"] = {"error": str(e)[-300:], "cores": allowed}
    else:
        out["full_host"] = {"value": None, "cores": allowed,
                            "limit": f"the job may use {allowed} cores (cgroup quota {quota}, "
                                     f"{phys} physical): the share run above is the full host "
                                     "available to it"}
    return out


def host_cpu_info():
    """CPU model, logical CPUs visible, physical cores and SMT state of this host."""
    info = {"model": None, "logical_cpus": os.cpu_count(), "physical_cores": None, "smt": None}
    try:
        cores = set()
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and info["model"] is None:
                info["model"] = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
            elif not k and phys is not None:
                cores.add((phys, core))
                phys = core = None
        if phys is not None:
            cores.add((phys, core))
        info["physical_cores"] = len(cores) or None
    except OSError:
        pass
    try:
        info["smt"] = open("/sys/devices/system/cpu/smt/active").read().strip() == "1"
    except OSError:
        pass
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    return info


def _grid_parts(O, g, n):
    """numpy copy of an oracle cell grid's (cell-ordered) struct part array."""
    from swift_subtask_dev_amd import abi

    ptr = O.fn("f32", "cellgrid_parts")(g)
    raw = (C.c_uint8 * (n * abi.PART_DTYPE.itemsize)).from_address(ptr)
    return abi.copy_parts(np.frombuffer(raw, dtype=np.uint8).view(abi.PART_DTYPE))


def parity_vs_cpu(ctx, parts, P, tuning, threads, workload="sedov"):
    """Outside the timed region: one density loop (after hydro_init_part) and
    one force loop (after hydro_reset_acceleration) on the bench's own input,
    on the GPU and in the CPU baseline's float port; max relative differences
    per output field, matched by particle id."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    import parity_bars as B
    from swift_subtask_dev_amd import abi, lib

    n = len(parts)
    bars = B.BARS["eagle" if workload == "eagle" else "sedov128"]
    eb = abi.EngineBundle(dim=tuple(P.dim), periodic=True, params=P, max_active_bin=P.max_active_bin)
    # GPU
    gd, gf = abi.copy_parts(parts), abi.copy_parts(parts)
    sp = lib.HydroSpace(ctx)
    sp.set_tuning(*tuning)
    sp.upload(gd)
    sp.rebuild(P)
    sp.init_parts(P)
    sp.density(P)
    sp.download(gd, abi.FIELDS_DENSITY)
    sp.upload(gf)
    sp.rebuild(P)
    sp.reset_acceleration(P)
    sp.force(P)
    sp.download(gf, abi.FIELDS_FORCE)
    sp.close()
    # CPU float port
    cd, cf = abi.copy_parts(parts), abi.copy_parts(parts)
    O.fn("f32", "init_parts")(cd.ctypes.data, n, C.byref(P))
    cf["a_hydro"] = 0
    cf["u_dt"] = 0
    cf["h_dt"] = 0
    cf["min_ngb_time_bin"] = abi.NUM_TIME_BINS + 1
    out, bar = {}, {}
    for arr, loop, fields in ((cd, 0, ("rho", "wcount", "wcount_dh", "rho_dh", "div_v")),
                              (cf, 2, ("a_hydro", "u_dt", "h_dt"))):
        g = O.fn("f32", "cellgrid_new")(arr.ctypes.data, n, float(P.dim[0]), 20)
        O.fn("f32", "cellgrid_run")(g, C.addressof(eb.runner), loop, threads)
        cpu = _grid_parts(O, g, n)
        O.fn("f32", "cellgrid_free")(g)
        gpu = gd if loop == 0 else gf
        cpu = cpu[np.argsort(cpu["id"], kind="stable")]
        gpu = gpu[np.argsort(gpu["id"], kind="stable")]
        for f in fields:
            a = gpu[f].astype(np.float64).reshape(n, -1)
            b = cpu[f].astype(np.float64).reshape(n, -1)
            floor = (1e-6 if loop == 0 else 1e-4) * max(np.abs(b).max(), 1e-300)
            out[f] = float((np.abs(a - b) / np.maximum(np.abs(b), floor)).max())
            if f in bars:  # the stated tolerance of tests/parity_bars.py
                mx, q = B.summary(gpu, cpu, (f,))[f]
                bar[f] = {"max": mx, "p99.9": q, "bar_max": bars[f][0], "bar_p99.9": bars[f][1],
                          "ok": bool(mx <= bars[f][0] and q <= bars[f][1])}
        if loop == 2:
            out["min_ngb_time_bin_equal"] = bool(np.array_equal(gpu["min_ngb_time_bin"],
                                                                cpu["min_ngb_time_bin"]))
    return {"vs": "cpu_baseline float port (same input, one density + one force loop)",
            "max_rel": out,
            "bars": bar,
            "bars_source": "tests/parity_bars.py (floor 1e-4 x the column maximum; the same "
                           "bars test_gpu_physics.py::test_baseline_chain_from_unconverged_vs_f32 "
                           "asserts on the whole chain)",
            "floor": "1e-6 (density fields) / 1e-4 (force fields) x the column maximum",
            "note": "GPU fp64 against the FLOAT port (the reference's own precision): the "
                    "differences are the port's float rounding (a_hydro ~1e-3 relative where "
                    "pressure-gradient terms cancel); against the f64 oracle the same loops "
                    "hold 2e-6 (density) / 5e-5 (force) with exact counts "
                    "(tests/test_gpu_parity.py, test_gpu_physics.py)"}


def chain_vs_f32(raw, gpu, gpu_counts, P, workload):
    """Outside the timed region: the setup's whole GPU chain (density, ghost,
    gradient, extra ghost, force, end force from the unconverged input)
    against the float restatement's chain on the same input, per field under
    the stated bars of tests/parity_bars.py -- the check
    test_gpu_physics.py::test_baseline_chain_from_unconverged_vs_f32 asserts."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    import parity_bars as B
    from swift_subtask_dev_amd import abi

    o = abi.copy_parts(raw)
    n = len(o)
    O.fn("f32", "init_parts")(o.ctypes.data, n, C.byref(P))
    counts = {"density": O.fn("f32", "box_density")(o.ctypes.data, n, C.byref(P), None)}
    nfail = C.c_longlong(0)
    O.fn("f32", "box_ghost")(o.ctypes.data, n, C.byref(P), C.byref(nfail))
    counts["gradient"] = O.fn("f32", "box_gradient")(o.ctypes.data, n, C.byref(P), None)
    O.fn("f32", "box_extra_ghost")(o.ctypes.data, n, C.byref(P))
    counts["force"] = O.fn("f32", "box_force")(o.ctypes.data, n, C.byref(P), None)
    O.fn("f32", "box_end_force")(o.ctypes.data, n, C.byref(P))
    bars = B.BARS["eagle" if workload == "eagle" else "sedov128"]
    res = {}
    for f, (mx, q) in B.summary(gpu, o, bars).items():
        res[f] = {"max": mx, "p99.9": q, "bar_max": bars[f][0], "bar_p99.9": bars[f][1],
                  "ok": bool(mx <= bars[f][0] and q <= bars[f][1])}
    cnt = {k: {"gpu": int(gpu_counts[k]), "f32": int(v),
               "ok": bool(abs(gpu_counts[k] - v) <= B.COUNT_REL * v)} for k, v in counts.items()}
    return {"vs": "liboracle_f32 whole chain (the reference's float arithmetic) from the same "
                  "unconverged input", "fields": res, "counts": cnt,
            "all_ok": all(r["ok"] for r in res.values()) and all(c["ok"] for c in cnt.values())}


def flow_vs_f32(ctx, n=64):
    """Outside the timed region: the terms the Sedov input (v = 0) leaves at
    zero -- the artificial viscosity of approaching pairs, the diffusion, the
    switch evolution -- on ics.flow_box(n) (converging, shearing flow, lumpy
    u): the GPU's whole chain against the float restatement's and the f64
    oracle's chains, under tests/parity_bars.py's flow64 bars (the check
    test_gpu_physics.py::test_flow_chain_vs_f32_and_f64 asserts)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    import parity_bars as B
    from swift_subtask_dev_amd import abi, ics, lib

    parts = ics.flow_box(n)
    P = abi.default_hydro_params((1.0, 1.0, 1.0), True)
    P.max_active_bin = 1
    g = abi.copy_parts(parts)
    sp = lib.HydroSpace(ctx)
    sp.upload(g)
    sp.rebuild(P)
    res = sp.hydro_step(P)
    sp.download(g, abi.FIELDS_ALL)
    sp.close()
    chains = {}
    for prec in ("f32", "f64"):
        o = abi.copy_parts(parts)
        N = len(o)
        O.fn("f32", "init_parts")(o.ctypes.data, N, C.byref(P))
        cnt = {"density": O.fn(prec, "box_density")(o.ctypes.data, N, C.byref(P), None)}
        nfail = C.c_longlong(0)
        O.fn(prec, "box_ghost")(o.ctypes.data, N, C.byref(P), C.byref(nfail))
        cnt["gradient"] = O.fn(prec, "box_gradient")(o.ctypes.data, N, C.byref(P), None)
        O.fn(prec, "box_extra_ghost")(o.ctypes.data, N, C.byref(P))
        cnt["force"] = O.fn(prec, "box_force")(o.ctypes.data, N, C.byref(P), None)
        O.fn(prec, "box_end_force")(o.ctypes.data, N, C.byref(P))
        chains[prec] = (o[np.argsort(o["id"], kind="stable")], cnt)
    g = g[np.argsort(g["id"], kind="stable")]
    (o32, c32), (o64, c64) = chains["f32"], chains["f64"]
    bars = B.BARS["flow64"]
    sg, so = B.summary(g, o32, bars), B.summary(o64, o32, bars)
    fields = {f: {"max": sg[f][0], "p99.9": sg[f][1], "bar_max": bars[f][0],
                  "bar_p99.9": bars[f][1], "f64_oracle_max": so[f][0], "f64_oracle_p99.9": so[f][1],
                  "ok": bool(sg[f][0] <= bars[f][0] and sg[f][1] <= bars[f][1]
                             and sg[f][0] <= 1.1 * so[f][0] + 1e-6
                             and sg[f][1] <= 1.1 * so[f][1] + 1e-6)} for f in bars}
    counts = {k: {"gpu": int(res[k]), "f32": int(c32[k]), "f64": int(c64[k]),
                  "ok": bool(abs(res[k] - c32[k]) <= B.COUNT_REL * c32[k] and res[k] == c64[k])}
              for k in ("density", "gradient", "force")}
    return {"vs": f"ics.flow_box({n}) (converging shearing flow: mu_ij < 0 viscosity, diffusion "
                  "and switches live): the GPU chain against liboracle_f32's chain (bars) and "
                  "liboracle_f64's (counts exact)",
            "viscous_heating_frac": float((o64["u_dt"] > 0).mean()),
            "fields": fields, "counts": counts,
            "all_ok": all(v["ok"] for v in fields.values()) and all(v["ok"] for v in counts.values())}


def step_breakdown(sp, P, stream, torch, local, reps=3):
    """Per-phase times of a whole SWIFT hydro step on the device-resident box,
    measured AFTER the timed region (not part of `value`): drift (drift_part +
    hydro_predict_extra), rebuild (re-bin + sort), then the SPHENIX chain. Two
    variants: rebuild every step, and drift-only (particles left in their
    cells, the loops' reach widened by dx_max). Velocities: v_full of |v| ~ 1
    with dt moving the fastest particle 0.1 h per step."""
    from swift_subtask_dev_amd import abi
    rng = np.random.Generator(np.random.PCG64(17))
    n = len(local)
    xp = abi.new_xparts(n)
    xp["v_full"] = rng.normal(0, 0.577, (n, 3)).astype(np.float32)
    sp.upload_xparts(xp)
    h = float(np.median(local["h"]))
    dt = 0.1 * h / float(np.abs(xp["v_full"]).max() * 1.733)
    # kicks and the thermal update on a CFL-limited step (the Sedov hot spot's
    # sound speed), positions moved by v_full over dt
    vsig = np.maximum(local["v_sig"].astype(np.float64), 1e-30)
    dt_cfl = min(dt, 0.1 * float(np.min(local["h"] / vsig)))
    D = abi.DriftParams(dt, dt_cfl, dt_cfl, dt_cfl, 0.0)
    sp.rebuild(P)
    sp.hydro_step(P)  # a consistent state (h_dt, u_dt of a whole chain) to drift from
    names = ["drift", "rebuild", "density", "ghost", "gradient", "extra_ghost", "force"]
    out = {}
    for mode in ("rebuild_every_step", "drift_only"):
        acc = {k: [] for k in names}
        dx = 0.0
        for _ in range(reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
            ev[0].record(stream)
            sp.drift(D, P)
            ev[1].record(stream)
            if mode == "rebuild_every_step":
                sp.rebuild(P)
            ev[2].record(stream)
            sp.init_parts(P)
            sp.density(P, count=False)
            ev[3].record(stream)
            sp.ghost(P)
            ev[4].record(stream)
            sp.gradient(P, count=False)
            ev[5].record(stream)
            sp.extra_ghost(P)
            ev[6].record(stream)
            sp.force(P, count=False)
            sp.end_force(P)
            ev[7].record(stream)
            torch.cuda.synchronize()
            for k, name in enumerate(names):
                acc[name].append(ev[k].elapsed_time(ev[k + 1]))
            dx = sp.info()["dx_max"]
        r = {f"{k}_ms": statistics.median(v) for k, v in acc.items()}
        r["step_ms"] = sum(r.values())
        r["dx_max_over_h"] = dx / h
        out[mode] = r
    out["note"] = ("untimed by the headline; medians of 3 steps; drift_only accumulates "
                   "dx_max over its 3 steps (0.1 h each); kicks on a CFL step")
    return out


def steady_state(sp, P, stream, torch, local, n_owned, args, skin=None, steps=None, disp=None):
    """K steps of drift + density + force on the device-resident box with the
    pair lists kept while valid (swh_tuning.list_keep). Drift velocities:
    random, |v| ~ 1, dt so that the fastest particle moves `disp` h_min per step
    (a Courant-limited subsonic flow moves < 0.05 h per step; with the smallest
    h, h_dt dt / h stays small for every particle, as SWIFT's time bins keep it,
    so the predicted h of a clustered box stays finite); the space is
    re-binned every `rebin` steps (dx bound > half a cell). The K steps run
    twice from the same state: counted (exact interactions per step), then
    timed without counting; the list builds the device ran are reported."""
    from swift_subtask_dev_amd import abi
    skin = args.steady_skin if skin is None else skin
    steps = args.steady_steps if steps is None else steps
    disp = args.steady_disp if disp is None else disp
    # Skin policy from the displacement per step: a list of skin s stays valid
    # while every particle's H + 2 dx_max <= its build reach H (1 + s), i.e.
    # ~kernel_gamma s / (2 disp) steps, and its walks grow as (1 + s)^3. A
    # list that cannot outlive two steps costs more than it saves: then every
    # density loop rebuilds with the headline's skin (no keep check).
    life = KERNEL_GAMMA * skin / (2.0 * disp)
    keep = 1
    policy = f"kept lists, skin {skin} (~{life:.2f} steps per build)"
    if life < 2.0:
        policy = (f"rebuild per step, skin {args.list_skin}: a skin-{skin} list would last "
                  f"{life:.2f} steps")
        skin, keep = args.list_skin, 0
    rng = np.random.Generator(np.random.PCG64(23))
    n = len(local)
    xp = abi.new_xparts(n)
    xp["v_full"] = rng.normal(0.0, 0.577, (n, 3)).astype(np.float32)
    vmax = float(np.sqrt((xp["v_full"].astype(np.float64) ** 2).sum(axis=1)).max())
    h = float(np.min(local["h"][:n_owned]))
    dt = disp * h / vmax
    D = abi.DriftParams(dt, 0.0, 0.0, 0.0, 0.0)
    sp.set_tuning(args.cell_factor, args.loop_variant, args.group_size, args.cell_scale, 0,
                  args.list_capacity, skin, keep)

    def reset():
        sp.upload(local)
        sp.set_owned(n_owned)
        sp.rebuild(P)
        sp.upload_xparts(xp)

    reset()
    w = min(sp.info()["cell_width"])
    rebin = max(1, int(args.steady_rebin * w / (vmax * dt)))

    per_step = []

    def run(count, ev=None):
        nd = nf = 0
        for k in range(steps):
            if k > 0 and k % rebin == 0:
                sp.rebuild(P)
            # hydro_reset_acceleration first: the drift's hydro_predict_extra
            # then sees h_dt = 0 and keeps h (this loop has no ghost, so the
            # force loop's h_dt comes from un-finalised densities and would
            # blow h up on a clustered box); the force loop still starts
            # from zeroed accumulators
            sp.reset_acceleration(P)
            sp.drift(D, P)
            sp.init_parts(P)
            if ev:
                ev[k][0].record(stream)
            r = sp.density(P, count=count)
            if ev:
                ev[k][1].record(stream)
                ev[k][2].record(stream)
            q = sp.force(P, count=count)
            if ev:
                ev[k][3].record(stream)
            if count:
                nd += r
                nf += q
                per_step.append((int(r), int(q)))
        return nd, nf

    b0 = sp.info()["list_builds"]
    nd, nf = run(True)
    builds = sp.info()["list_builds"] - b0
    reset()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
    t0 = time.perf_counter()
    run(False, ev)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    td = statistics.mean([e[0].elapsed_time(e[1]) for e in ev])
    tf = statistics.mean([e[2].elapsed_time(e[3]) for e in ev])
    b_d = n_owned * (27 * S_IN_DENSITY + S_OUT_DENSITY)
    return {"note": "untimed by the headline: drift + density + force per step with the pair "
                    "lists kept across drifts while valid (device check, rebuilt on the device "
                    "when a particle's H + 2 D exceeds its build reach)",
            "steps": steps, "list_skin": skin, "skin_policy": policy,
            "displacement_per_step_over_h": disp,
            "h_during_drift": "frozen: each step resets the accelerations (h_dt = 0) before its "
                              "drift, so hydro_predict_extra keeps h and only positions move "
                              "(this loop has no ghost to finalise h_dt)",
            "rebin_every": rebin, "list_builds": int(builds),
            "steps_per_list_build": steps / max(1, builds),
            "interactions": nd + nf, "ms_per_step": el / steps * 1e3,
            "interactions_first_last_step": [per_step[0], per_step[-1]] if per_step else None,
            "interactions_per_s": (nd + nf) / el,
            "density_ms": td, "force_ms": tf,
            "density_roofline_frac": b_d / (td * 1e-3) / HBM_PEAK}


def load_traffic(workload="sedov"):
    """PMC-measured HBM bytes of the roofline kernel(s), per workload
    (profiles/traffic_density.json: Sedov 128^3 density loop;
    profiles/traffic_<workload>.json otherwise)."""
    name = "traffic_density.json" if workload == "sedov" else f"traffic_{workload}.json"
    path = ROOT / "profiles" / name
    if path.exists():
        try:
            return json.loads(path.read_text())
        except Exception:
            return None
    return None


def run_grav(args, ctx, rank, world, dist, torch):
    """BASELINE config 4: GravityTests uniform DM box, P2P leaf interactions
    (runner_doself_grav_pp + runner_dopair_grav_pp over each leaf and its 26
    neighbours, the near field a tree walk leaves to P2P), fp64. n^3 uniform
    gparts (Gravity_glass/makeIC.py: L = 1, rho = 1), softening 0.001
    (uniform_DM_box.yml), leaves of <= 400 gparts (space_splitsize). With
    N ranks the i-leaves are split into N contiguous ranges (strong split of
    the one box; gparts replicated read-only)."""
    from swift_subtask_dev_amd import abi, ics, lib

    n = args.n
    t0 = time.time()
    gp = ics.uniform_gravity_box(n, epsilon=0.001, seed=256)
    cdim = int(np.ceil((n ** 3 / 400.0) ** (1.0 / 3.0)))
    gs, leaves = ics.leaf_cells(gp, cdim)
    del gp
    offs, pairs = ics.neighbour_pairs(cdim, periodic=False, truncated=0)
    nl = len(leaves)
    lo, hi = rank * nl // world, (rank + 1) * nl // world
    if world > 1:  # this rank's i-leaves keep their source lists, the others none
        own = np.zeros(nl + 1, dtype=np.int64)
        own[lo + 1:hi + 1] = np.diff(offs)[lo:hi]
        sel = np.concatenate([np.arange(offs[k], offs[k + 1]) for k in range(lo, hi)])
        pairs = pairs[sel]
        offs = np.cumsum(own).astype(np.int32)
    G = abi.GravParams(0, (C.c_float * 3)(1, 1, 1), 0.0, 1e30, abi.NUM_TIME_BINS)
    sp = lib.GravSpace(ctx)
    stream = torch.cuda.Stream()
    sp.upload(gs)
    sp.set_leaves(leaves, offs, pairs)
    n_int = sp.pp(G)
    torch.cuda.synchronize()
    log(f"[rank {rank}] grav setup {time.time() - t0:.1f}s: {len(gs)} gparts, {nl} leaves "
        f"(cdim {cdim}, max {int(leaves['count'].max())}), {n_int} P2P interactions/step")
    for _ in range(args.warmup):
        sp.pp(G, count=False)
    sp.sync()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        sp.pp(G, count=False)
    sp.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    tot = torch.tensor([float(n_int) * args.steps], dtype=torch.float64, device=RED_DEVICE)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=RED_DEVICE)
    if dist:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    total, el = tot.item(), tmax.item()
    if rank == 0:
        flops = total * 28.0 / el  # P2P Newtonian 28 flops per interaction
        out = {
            "metric": "P2P gravity interactions/s (runner_doself/dopair_grav_pp near field), "
                      f"uniform DM box {n}^3",
            "value": total / el, "unit": "interactions/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (uniform random gparts, seed 256; Gravity_glass ICs unavailable offline)",
            "config": {"workload": f"GravityTests uniform DM box {n}^3: leaf self + 26 neighbour "
                                   "leaf pairs, P2P, softening 0.001, non-periodic",
                       "gparts": int(len(gs)), "leaves": nl, "leaf_cdim": cdim,
                       "interactions_per_step": int(total / args.steps)},
            "roofline": {"bound": "fp64-vector", "kernel": "p2p_kernel", "achieved": flops / 1e12,
                         "peak": FP64_PEAK / 1e12, "unit": "TFLOP/s", "frac": flops / FP64_PEAK,
                         "traffic": None, "flops_model": "28 flops per directed P2P interaction"},
            "cpu_baseline": None,
        }
        tr = load_traffic("grav") if (n == 256 and world == 1) else None
        if tr:
            out["roofline"]["traffic"] = tr.get("bytes_per_launch")
            out["roofline"]["traffic_source"] = tr.get("source")
            out["roofline"]["traffic_commit"] = tr.get("commit")
        if world == 1 and not args.no_cpu_baseline:
            try:
                # bounded sample: the first 1% of the i-leaves with their full
                # source lists (every leaf stays a source)
                k = max(1, nl // 100)
                so = np.zeros(nl + 1, dtype=np.int32)
                so[1:k + 1] = np.diff(offs)[:k]
                so = np.cumsum(so).astype(np.int32)
                threads = cpu_share_threads()
                w = run_cpu_worker("grav", {"gparts": np.ascontiguousarray(gs).view(np.uint8),
                                            "leaves": leaves, "offs": so,
                                            "pairs": pairs[:so[-1]],
                                            "G": np.frombuffer(bytes(G), dtype=np.uint8)},
                                   {"runs": 2}, threads)
                out["cpu_baseline"] = {
                    "value": w["interactions"] / w["seconds_share"], "unit": "interactions/s",
                    "cores": threads, "kind": "port", "host": host_cpu_info(),
                    "pinning": "one thread per physical core, child process without torch",
                    "sample": f"the first {k} of {nl} i-leaves with their 27-leaf source "
                              f"lists: {w['interactions']} P2P interactions, float "
                              f"restatement of runner_doself/dopair_grav_pp, median of 2 runs "
                              f"after 1 warm-up ({w['seconds_share']:.3f} s)"}
                out["gpu_over_cpu"] = out["value"] / out["cpu_baseline"]["value"]
            except Exception as e:  # report, never fake
                log(f"grav cpu baseline failed: {e}")
        print(json.dumps(out), flush=True)
    sp.close()


def run_cosmo(args, ctx, rank, world, dist, torch):
    """BASELINE config 5 stand-in: SmallCosmoVolume hydro + self-gravity
    (small_cosmo_volume.yml), its first step. ics.small_cosmo_volume(64): a
    Zel'dovich 64^3 DM field split into DM + gas as space_generate_gas does
    (src/space.c:1747-1935), box units of 142.248 Mpc, km/s, G = 1; WMAP9
    cosmology at a = 0.0198 (cosmo.small_cosmo_volume_params: the hydro loops
    take a, H, a^2 H and the gamma = 5/3 scale-factor powers); softening 1/25
    of the mean separation, PM mesh 64, a_smooth 1.25, r_cut_max 4.5 r_s,
    theta_cr 0.7, cell_split_size 50, and the yml's MAC: adaptive with
    epsilon_fmm 0.001 (gravity_M2L_accept, src/multipole_accept.h:81-170),
    fed |a_tree + a_mesh / G| of an untimed geometric-MAC step as SWIFT's
    gravity_end_force records old_a_grav_norm
    (src/gravity/MultiSoftening/gravity.h:244-253). SWH_COSMO_MAC=geometric
    times the theta_cr-only walk instead.

    One step = the hydro density + force loops on the gas and the gravity of
    every gpart: the recursive gravity tasks over the cell tree (P2P, M2P,
    M2L, L2L, L2P) plus the PM mesh. Hydro is queued on its own stream, then
    the gravity chain runs on the high-priority gravity stream (the two task
    families of a SWIFT step overlap); the line reports each alone and both.

    With N ranks (one per GPU) the step is sharded: the gas by the
    hydro block decomposition (decomp.HaloPlan: owned block + read-only halo,
    swh_space_set_owned) with the halo's rho refreshed point-to-point between
    density and force (decomp.DeviceHalo, as the sedov step), the gravity by
    subtrees of the top cells whose centres lie in the rank's block
    (decomp.gravity_owned_cells, swh_gspace_set_owned_cells) with every gpart
    and the tree replicated read-only, and the PM mesh computed by every rank
    on its replicated gparts. value = interactions of all ranks / the slowest
    rank's time."""
    import threading
    from swift_subtask_dev_amd import abi, cosmo, decomp, ics, lib

    n = args.n if args.n != 128 else 64
    box = (1.0, 1.0, 1.0)
    t0 = time.time()
    gas, gp = ics.small_cosmo_volume(n)
    cm, P = cosmo.small_cosmo_volume_params()
    gas["time_bin"] = cosmo.SCV_FIRST_BIN
    sp = lib.HydroSpace(ctx)
    sp.upload(gas)
    sp.rebuild(P)
    chain = sp.hydro_step(P)  # converged h, the force inputs (whole box, untimed)
    sp.download(gas, abi.FIELDS_ALL)
    sp.close()
    eps = 1.0 / (25.0 * n)
    N_mesh = 64
    r_s = 1.25 / N_mesh
    mac = os.environ.get("SWH_COSMO_MAC", "adaptive")
    G = abi.GravParams(1, (C.c_float * 3)(1, 1, 1), 1.0 / r_s, 0.1 * r_s, abi.NUM_TIME_BINS)
    G.theta_crit = 0.7
    G.adaptive_tolerance = 1e-3
    G.r_cut_max = 4.5 * r_s
    g, cells, tops = ics.gravity_tree(gp, 8, split_size=50)
    pairs = ics.top_level_pairs(tops)
    gs = lib.GravSpace(ctx)
    # an untimed geometric-MAC step gives the adaptive MAC its |a| estimate:
    # old_a_grav_norm = |a_tree + a_mesh / G| (gravity.h:244-253), G = 1
    gs.upload(g)
    gs.set_tree(cells)
    G.use_advanced_MAC = 0
    gs.tree(G, tops, pairs)
    gs.pm_mesh(N_mesh, 1.0, r_s, 1.0)
    g0 = abi.copy_parts(g)
    gs.download(g0)
    g["old_a_grav_norm"] = np.linalg.norm(g0["a_grav"].astype(np.float64)
                                          + g0["a_grav_mesh"].astype(np.float64), axis=1)
    G.use_advanced_MAC = 1 if mac == "adaptive" else 0
    gs.upload(g)
    gs.set_tree(cells)
    owned_cells = None
    if world > 1:
        owned_cells = decomp.gravity_owned_cells(cells, tops, rank, world, box)
        gs.set_owned_cells(owned_cells)
    stats = gs.tree(G, tops, pairs)
    gs.pm_mesh(N_mesh, 1.0, r_s, 1.0)

    hs = lib.HydroSpace(ctx)
    hstream = torch.cuda.Stream()
    hs.set_stream(hstream.cuda_stream)
    plan = None
    if world > 1:
        reach = 1.01 * KERNEL_GAMMA * float(gas["h"].max())  # 1.01 gamma h_max, as the sedov split
        plan = decomp.HaloPlan(gas["x"], box, world, rank, reach)
        local, n_owned = plan.local_set(gas), plan.n_owned
    else:
        local, n_owned = gas, len(gas)
    hs.upload(local)
    hs.set_owned(n_owned)
    hs.rebuild(P)
    exchanger = decomp.DeviceHalo(plan, hs, dist, torch, hstream) if plan else None
    hs.init_parts(P)
    n_density = hs.density(P)
    hs.reset_acceleration(P)
    n_force = hs.force(P)
    torch.cuda.synchronize()
    log(f"[rank {rank}] cosmo setup {time.time() - t0:.1f}s: {n_owned} of {n ** 3} gas + "
        f"{2 * n ** 3} gparts ({int(owned_cells.sum()) if owned_cells is not None else len(cells)}"
        f" of {len(cells)} cells owned); a = {P.a:.5f}, H = {P.H:.4g}; chain {chain}; "
        f"gravity step ({mac} MAC) {stats}; hydro {n_density} + {n_force}")

    def hydro_async():
        hs.init_parts(P)
        hs.density(P, count=False)
        if exchanger:  # the force loop reads the neighbours' new rho
            exchanger.refresh(abi.HALO_RHO)
        hs.reset_acceleration(P)
        hs.force(P, count=False)

    def hydro():
        hydro_async()
        hs.sync()

    def gravity():
        gs.tree(G, tops, pairs, stats=False)  # the device accumulators restart at every walk
        gs.pm_mesh(N_mesh, 1.0, r_s, 1.0)
        gs.sync()

    overlap = os.environ.get("SWH_COSMO_OVERLAP", "async")

    def both():
        if overlap == "thread":  # hydro from a second host thread
            th = threading.Thread(target=gravity)
            th.start()
            hydro()
            th.join()
        else:
            # one host thread: the gravity chain (the step's critical path) is
            # queued first on its high-priority stream -- the tree walk's levels
            # return to the host, then the P2P and M2P are queued -- and the
            # hydro loops are queued on their own stream behind it (no host
            # wait), filling the CUs the chain leaves idle
            gs.tree(G, tops, pairs, stats=False)
            hydro_async()
            gs.pm_mesh(N_mesh, 1.0, r_s, 1.0)
            gs.sync()
            hs.sync()

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        t = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        if dist:
            dist.barrier()
            x = torch.tensor([el], dtype=torch.float64, device=RED_DEVICE)
            dist.all_reduce(x, op=dist.ReduceOp.MAX)
            el = x.item()
        return el / args.steps

    t_h, t_g, t_b = timed(hydro), timed(gravity), timed(both)
    mine = [float(n_density + n_force + stats["n_pp"]), float(n_density + n_force),
            float(stats["n_pp"])]
    tot = torch.tensor(mine, dtype=torch.float64, device=RED_DEVICE)
    if dist:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    total, total_hydro, total_pp = tot.tolist()
    # roofline: the step's dominant kernel is the gravity P2P (its own HIP
    # events inside swh_grav_tree, on the gravity stream)
    st = gs.tree(G, tops, pairs)
    gs.sync()
    if rank == 0:
        out = {
            "metric": "hydro (density+force) + gravity P2P interactions/s, SmallCosmoVolume stand-in",
            "value": total / t_b, "unit": "interactions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": t_b * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (Zel'dovich 64^3 DM field split into DM + gas as space_generate_gas, "
                    "z = 50; SmallCosmoVolume ICs unavailable offline)",
            "config": {"workload": f"SmallCosmoVolume stand-in: {n}^3 gas + {n}^3 DM, first step "
                                   f"(a = {P.a:.5f}): hydro density + force loops || gravity tree "
                                   f"(P2P, M2P, M2L, L2L, L2P; {mac} MAC) + PM mesh 64",
                       "parallelism": (f"{'x'.join(map(str, decomp.block_dims(world)))} blocks: gas "
                                       "owned + halo (rho refreshed between density and force), "
                                       "gravity subtrees owned, gparts replicated"
                                       if world > 1 else "one GPU"),
                       "ranks": RANKS,
                       "cosmology": {"a": P.a, "H": P.H, "Omega_cdm": ics.SCV_OMEGA_CDM,
                                     "Omega_b": ics.SCV_OMEGA_B, "Omega_lambda": ics.SCV_OMEGA_L,
                                     "units": "box (142.248 Mpc), km/s, G = 1"},
                       "mac": {"kind": mac, "theta_crit": 0.7, "epsilon_fmm": 1e-3,
                               "old_a_grav_norm": "|a_tree + a_mesh/G| of an untimed geometric step"},
                       "hydro_interactions_per_step": int(total_hydro),
                       "gravity_pp_per_step": int(total_pp),
                       "gravity_tree_stats_rank0": stats, "cells": int(len(cells)),
                       "softening": eps, "r_s": r_s},
            "step_ms": {"hydro_alone": t_h * 1e3, "gravity_alone": t_g * 1e3,
                        "overlapped": t_b * 1e3,
                        "overlap_gain": (t_h + t_g) / t_b, "overlap_mode": overlap},
            "gravity_phase_ms_rank0": st["ms"],
            "roofline": None, "cpu_baseline": None,
        }
        t_p2p = st["ms"]["p2p"] * 1e-3
        if t_p2p > 0:
            # 28 flops per Newtonian pair, 43 per truncated pair
            n_tr = st["n_pp_truncated"]
            flops = ((st["n_pp"] - n_tr) * 28.0 + n_tr * 43.0) / t_p2p
            out["roofline"] = {"bound": "fp64-vector", "kernel": "p2p_batch_kernel (small leaves; p2p_kernel for leaves > 64)",
                               "achieved": flops / 1e12, "peak": FP64_PEAK / 1e12,
                               "unit": "TFLOP/s", "frac": flops / FP64_PEAK, "traffic": None,
                               "flops_model": f"SURVEY 8d: 43 flops per truncated P2P pair "
                                              f"({n_tr} of {st['n_pp']}), 28 per Newtonian pair",
                               "pp_truncated": int(n_tr)}
            tr = load_traffic("cosmo") if world == 1 else None
            if tr:
                out["roofline"]["traffic"] = tr.get("bytes_per_launch")
                out["roofline"]["traffic_source"] = tr.get("source")
                out["roofline"]["traffic_commit"] = tr.get("commit")
        if world == 1 and not args.no_cpu_baseline:
            try:
                threads = cpu_share_threads()
                w = run_cpu_worker("cosmo", {"parts": np.ascontiguousarray(gas).view(np.uint8),
                                             "gparts": np.ascontiguousarray(g).view(np.uint8),
                                             "cells": np.ascontiguousarray(cells).view(np.uint8),
                                             "tops": np.ascontiguousarray(tops, dtype=np.int32),
                                             "pairs": np.ascontiguousarray(pairs, dtype=np.int32)
                                             .reshape(-1),
                                             "G": np.frombuffer(bytes(G), dtype=np.uint8)},
                                   {"cdim": 20}, threads)
                n_cpu = n_density + n_force + w["tree_stats"][0]
                out["cpu_baseline"] = {
                    "value": n_cpu / w["seconds_share"], "unit": "interactions/s",
                    "cores": threads, "kind": "port", "host": host_cpu_info(),
                    "pinning": "one thread per physical core, child process without torch",
                    "sample": f"one whole step, the same inputs and MAC: the float restatement's "
                              f"density + force loops over a cdim-20 cell grid "
                              f"({w['seconds_hydro']:.2f} s, OpenMP over cells) and its gravity "
                              f"({w['seconds_gravity']:.2f} s): P2M/M2M per tree depth, the "
                              f"recursive self/pair tasks in chunks of 64 over the threads (as "
                              f"SWIFT's runners run them, runner_main.c:207-208, 257-258), "
                              f"P2P/M2P and M2L over target cells, L2L per depth and L2P over "
                              f"leaves, all OpenMP on the same threads; the PM mesh not "
                              f"included (the GPU step's value includes it)",
                    "tree_stats": w["tree_stats"]}
                out["gpu_over_cpu"] = out["value"] / out["cpu_baseline"]["value"]
            except Exception as e:  # report, never fake
                log(f"cosmo cpu baseline failed: {e}")
        print(json.dumps(out), flush=True)
    hs.close()
    gs.close()


# BASELINE.json configs 3-5, run after the headline by the default 1-GPU
# bench (bench.py --workload ...): each child prints one JSON line with its
# own value, ms_per_step, roofline (the PMC traffic named by commit) and
# cpu_baseline
OTHER_CONFIGS = {
    "config3_eagle": ["--workload", "eagle"],
    "config4_grav256": ["--workload", "grav", "--n", "256"],
    "config5_cosmo": ["--workload", "cosmo"],
}


def other_configs(args):
    import subprocess

    res = {}
    for name, extra in OTHER_CONFIGS.items():
        cmd = [sys.executable, str(Path(__file__).resolve()), *extra, "--steps", str(args.steps),
               "--warmup", str(args.warmup), "--no-configs"]
        if args.no_cpu_baseline:
            cmd.append("--no-cpu-baseline")
        t0 = time.perf_counter()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=400)
            sys.stderr.write(r.stderr[-4000:])
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not lines:
                res[name] = {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-800:]}
            else:
                res[name] = json.loads(lines[-1])
        except Exception as e:  # report, never fake
            res[name] = {"error": str(e)[-300:]}
        res[name]["command"] = " ".join(["python", "bench.py", *cmd[2:]])
        res[name]["wall_s"] = time.perf_counter() - t0
        log(f"{name}: {res[name].get('value')} {res[name].get('unit', '')} "
            f"({res[name]['wall_s']:.0f} s)")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=128, help="particles per dimension per GPU")
    ap.add_argument("--cell-factor", type=int, default=int(os.environ.get("SWH_CELL_FACTOR", "1")))
    ap.add_argument("--loop-variant", type=int, default=0, choices=[0, 7],
                    help="0 default (7): pair lists")
    ap.add_argument("--cell-scale", type=float, default=float(os.environ.get("SWH_CELL_SCALE", "0")),
                    help="grid cells per H_max as a real number (overrides --cell-factor)")
    ap.add_argument("--diag-mode", type=int, default=0,
                    help="profiling only, results invalid: 1 tile staging only, 2 + candidate tests")
    ap.add_argument("--group-size", type=int, default=int(os.environ.get("SWH_GROUP_SIZE", "0")),
                    help="tile i-group size / row width: 0 (default 16), 16, 32, 64")
    ap.add_argument("--list-skin", type=float, default=float(os.environ.get("SWH_LIST_SKIN", "0.01")),
                    help="pair-list reach slack over gamma*h (the library default, "
                         "SWH_DEFAULT_LIST_SKIN = 0.01)")
    ap.add_argument("--list-capacity", type=int, default=0, help="pair-list entries per particle")
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-runs", type=int, default=3)
    ap.add_argument("--no-steady", action="store_true", help="skip the untimed steady-state run")
    ap.add_argument("--steady-skin", type=float, default=0.1)
    ap.add_argument("--steady-steps", type=int, default=24)
    ap.add_argument("--steady-rebin", type=float, default=0.25,
                    help="re-bin the space once the fastest particle can have moved this many cell widths")
    ap.add_argument("--steady-disp", type=float, default=0.05,
                    help="steady state: displacement of the fastest particle per step / h")
    ap.add_argument("--no-breakdown", action="store_true",
                    help="skip the untimed full-step breakdown (drift, rebuild, chain)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the BASELINE configs 3-5 lines the default 1-GPU run appends "
                         "(each a child bench.py run, untimed by the headline)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: the 128^3 box split over the GPUs (the metric); "
                         "weak: one 128^3 box per GPU")
    ap.add_argument("--cpu-worker", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-input", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-meta", default="{}", help=argparse.SUPPRESS)
    ap.add_argument("--workload", default="sedov", choices=["sedov", "grav", "eagle", "cosmo"],
                    help="sedov: the headline metric (SedovBlast_3D 128^3 density + force); "
                         "grav: BASELINE config 4 (uniform DM box P2P, --n 256); "
                         "eagle: BASELINE config 3 stand-in (clustered box); "
                         "cosmo: BASELINE config 5 stand-in (hydro + tree/PM gravity, overlapped)")
    args = ap.parse_args()
    if args.cpu_worker:  # child of run_cpu_worker: no torch, no GPU
        cpu_worker_main(args.cpu_worker, args.cpu_input, json.loads(args.cpu_meta))
        return

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N`: one rank per GPU under torch.distributed.run,
        # started before anything here touches a GPU; exit with its code
        import socket
        import subprocess

        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
               f"--master-port={port}", str(Path(__file__).resolve())] + sys.argv[1:]
        log(f"launching {args.gpus} ranks: {' '.join(cmd)}")
        sys.exit(subprocess.call(cmd))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU")

    import torch

    # one rank per GPU; SWH_BENCH_BACKEND=gloo rehearses the multi-rank path
    # with several ranks sharing the GPUs there are (halo buffers staged
    # through the host) -- the driver's runs use RCCL, one GPU per rank
    global RED_DEVICE
    backend = os.environ.get("SWH_BENCH_BACKEND", "nccl")
    RED_DEVICE = "cuda" if backend == "nccl" else "cpu"  # gloo reduces host tensors
    device = local_rank % max(1, torch.cuda.device_count()) if backend == "gloo" else local_rank
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    from swift_subtask_dev_amd import abi, decomp, ics, lib

    # which GPU every rank drives (so a multi-GPU line shows its rank layout)
    global RANKS
    devs = [device]
    if dist:
        t = torch.tensor([device], dtype=torch.int64, device=RED_DEVICE)
        got = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(got, t)
        devs = [int(x.item()) for x in got]
    RANKS = {"world_size": dist.get_world_size() if dist else 1,
             "backend": dist.get_backend() if dist else None,
             "device_of_rank": devs, "visible_devices": torch.cuda.device_count()}

    if args.workload in ("grav", "cosmo"):
        ctx = lib.Context(device, args.precision)
        (run_grav if args.workload == "grav" else run_cosmo)(args, ctx, rank, world, dist, torch)
        ctx.close()
        if dist:
            dist.destroy_process_group()
        return

    n = args.n
    t_setup = time.time()
    strong = args.scaling == "strong"
    nslab = 1 if strong else world
    eagle = args.workload == "eagle"
    if eagle:
        # EAGLE_6 stand-in: 94^3 background + 64 Plummer clumps of
        # 13,000 (2 x 94^3-order gas particles, h spanning ~10x after the ghost)
        if not strong:
            raise SystemExit("--workload eagle runs one box (--scaling strong)")
        parts = ics.clustered_box(94, n_clumps=64, per_clump=13000, seed=6)
        box = (1.0, 1.0, 1.0)
    else:
        parts = ics.sedov_slabs(n, nslab)
        box = (float(nslab), 1.0, 1.0)
    P = abi.default_hydro_params(box, True)
    P.max_active_bin = 1
    ctx = lib.Context(device, args.precision)

    # ---- untimed setup: the full SPHENIX chain on the whole box ----------
    sp = lib.HydroSpace(ctx)
    sp.set_tuning(args.cell_factor, list_capacity=args.list_capacity, list_skin=args.list_skin)
    # the parity leg's chain check starts from the same unconverged input
    raw = abi.copy_parts(parts) if (world == 1 and not args.no_cpu_baseline) else None
    sp.upload(parts)
    sp.rebuild(P)
    chain = sp.hydro_step(P)
    sp.download(parts, abi.FIELDS_ALL)
    sp.close()
    chain_gpu = abi.copy_parts(parts) if raw is not None else None
    if eagle:  # converged h: re-bin on the final smoothing lengths
        log(f"[rank {rank}] eagle stand-in: {len(parts)} parts, h {parts['h'].min():.3g}.."
            f"{parts['h'].max():.3g}, chain ghost iterations {chain['ghost_iterations']}")
    hmax = float(parts["h"].max()) * KERNEL_GAMMA

    if strong:
        # one box, world blocks (2x2x2 at 8 GPUs); halo = everything within
        # gamma h_max of the block (decomp.py)
        plan = decomp.HaloPlan(parts["x"], box, world, rank, 1.01 * hmax)
        local, n_owned = plan.local_set(parts), plan.n_owned
    else:
        plan = None
        local, n_owned = decomp.slab_local_set(parts, rank, world, box[0], 1.02 * hmax,
                                               halo_time_bin=None)
    del parts
    sp = lib.HydroSpace(ctx)
    sp.set_tuning(args.cell_factor, args.loop_variant, args.group_size, args.cell_scale,
                  args.diag_mode, args.list_capacity, args.list_skin)
    # a dedicated (non-NULL) stream: the library's kernels, the halo exchange
    # and the timing events share it, so the events bracket exactly the loops
    stream = torch.cuda.Stream()
    sp.set_stream(stream.cuda_stream)
    sp.upload(local)
    sp.set_owned(n_owned)
    sp.rebuild(P)
    exchanger = decomp.DeviceHalo(plan, sp, dist, torch, stream) if plan and world > 1 else None
    # exact interaction counts of one step (same work every step: h is fixed)
    sp.init_parts(P)
    n_density = sp.density(P)
    stats_density = list(sp.info()["loop_stats"])
    sp.reset_acceleration(P)
    n_force = sp.force(P)
    stats_force = list(sp.info()["loop_stats"])
    torch.cuda.synchronize()
    info = sp.info()
    log(f"[rank {rank}] grid {info}")
    log(f"[rank {rank}] setup {time.time() - t_setup:.1f}s: {n_owned} owned + "
        f"{len(local) - n_owned} halo parts, {n_density} density + {n_force} force "
        f"interactions/step, chain ghost iterations {chain['ghost_iterations']}")

    def step(ev=None):
        sp.init_parts(P)
        if ev:
            ev[0].record(stream)
        sp.density(P, count=False)
        if ev:
            ev[1].record(stream)
        if exchanger:  # the force loop reads the neighbours' new rho
            exchanger.refresh(abi.HALO_RHO)
        if ev:
            ev[4].record(stream)
        sp.reset_acceleration(P)
        if ev:
            ev[2].record(stream)
        sp.force(P, count=False)
        if ev:
            ev[3].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t_dens = [e[0].elapsed_time(e[1]) * 1e-3 for e in events]
    t_force = [e[2].elapsed_time(e[3]) * 1e-3 for e in events]
    # the halo refresh of rho (pack, point-to-point swap, unpack) per rank
    halo = None
    if plan is not None and world > 1:
        rec_b = abi.HALO_RECORD_FLOATS * 4
        mine = {"rank": rank, "owned": int(n_owned), "halo": int(len(local) - n_owned),
                "peers": len(plan.peers()),
                "records_sent": int(sum(len(v) for v in plan.send.values())),
                "records_received": int(sum(c for _, c in plan.recv.values())),
                "record_bytes": rec_b,
                "exchange_ms": statistics.mean(e[1].elapsed_time(e[4]) for e in events)}
        halo = [None] * world
        dist.all_gather_object(halo, mine)

    tot = torch.tensor([float(n_density + n_force) * args.steps, float(n_owned)],
                       dtype=torch.float64, device=RED_DEVICE)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=RED_DEVICE)
    if dist:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    total_interactions, total_owned = tot.tolist()
    elapsed_max = tmax.item()
    # Steady state (untimed by the headline, which builds the lists in every
    # density loop): K x (drift + hydro_init_part + density + reset + force)
    # with the pair lists kept across drifts while their skin covers the
    # displacement (list_keep; the device decides and rebuilds), the space
    # re-binned every `rebin` steps -- SWIFT's step, which keeps its sorts
    # until the particles have moved too far.
    steady = None
    if world == 1 and args.diag_mode == 0 and not args.no_steady:
        try:
            steady = steady_state(sp, P, stream, torch, local, n_owned, args)
            # Where keeping the lists pays: a kept list of skin s stays valid for
            # ~gamma s / (2 disp) steps while its walks grow as (1 + s)^3, so at
            # the 0.05 h / step above every skin loses to a rebuild per step (the
            # policy in steady_state then rebuilds); at 0.01 h / step a 5% skin
            # lasts ~4-5 steps for ~16% more entries.
            steady["low_velocity"] = steady_state(sp, P, stream, torch, local, n_owned, args,
                                                  skin=0.05, disp=0.01)
        except Exception as e:  # report, never fake
            log(f"steady state failed: {e}")
        sp.set_tuning(args.cell_factor, args.loop_variant, args.group_size, args.cell_scale,
                      args.diag_mode, args.list_capacity, args.list_skin)
        sp.upload(local)
        sp.set_owned(n_owned)
        sp.rebuild(P)
    breakdown = None
    if world == 1 and not args.no_breakdown and not eagle:
        try:
            breakdown = step_breakdown(sp, P, stream, torch, local)
        except Exception as e:  # report, never fake
            log(f"step breakdown failed: {e}")

    if rank == 0:
        td = statistics.mean(t_dens)
        tf = statistics.mean(t_force)
        b_dens = n_owned * (27 * S_IN_DENSITY + S_OUT_DENSITY)
        b_force = n_owned * (27 * S_IN_FORCE + S_OUT_FORCE)
        achieved = b_dens / td
        # PMC traffic was measured on the default configuration only
        default_cfg = (args.loop_variant == 0 and args.group_size == 0 and args.list_skin == 0.01
                       and args.cell_factor == 1 and args.cell_scale == 0 and args.n == 128
                       and world == 1)
        traffic = load_traffic(args.workload) if default_cfg else None
        out = {
            "metric": METRIC_EAGLE if eagle else METRIC,
            "value": total_interactions / elapsed_max,
            "unit": "interactions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64" if args.precision == "f64" else "f32",
            "data": ("synthetic (EAGLE_6 stand-in: perturbed 94^3 lattice + 64 Plummer clumps of "
                     "13,000, h from the ghost; EAGLE ICs unavailable offline)" if eagle else
                     "synthetic (SedovBlast_3D-like perturbed lattice, eta=1.2348; glass IC "
                     "unavailable offline)"),
            "config": {
                "workload": (f"EAGLE_6 stand-in ({int(total_owned)} gas parts, clustered) split "
                             f"over {world} GPU(s)" if eagle else
                             f"SedovBlast_3D {n}^3 split over {world} GPU(s)" if strong else
                             f"SedovBlast_3D {n}^3 per GPU") +
                            ": density + force loops (SPHENIX, cubic spline)",
                "particles_per_gpu": n_owned,
                "global_particles": int(total_owned),
                "decomposition": (f"{'x'.join(map(str, decomp.block_dims(world)))} blocks + "
                                  "read-only halo, halo rho refreshed point-to-point "
                                  "between density and force"
                                  if strong else
                                  f"{world} x-slab(s) + read-only halo, no data-path collective"),
                "density_interactions_per_step": n_density,
                "force_interactions_per_step": n_force,
                "cell_factor": args.cell_scale or args.cell_factor,
                "loop_variant": args.loop_variant,
                "group_size": args.group_size or 16,
                "list_skin": args.list_skin,
                "list_entries": info["list_entries"],
                "list_overflow": info["list_overflow"],
                "grid_cdim": info["cdim"],
                "i_groups": info["ngroups"],
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "list_build_kernel + density_walk_kernel<double>",
                "achieved": achieved / 1e9,
                "peak": HBM_PEAK / 1e9,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK,
                "traffic": traffic.get("bytes_per_launch") if traffic else None,
                # PMC-measured HBM bytes of one density loop's kernels, from the
                # committed profile named here (not re-measured by this run)
                "traffic_source": (traffic.get("source", "profiles/traffic_density.json")
                                   if traffic else None),
                "traffic_commit": traffic.get("commit") if traffic else None,
                "bytes_model": f"N*(27*{S_IN_DENSITY}+{S_OUT_DENSITY}) = {b_dens} B per launch",
                "launch_ms": td * 1e3,
            },
            "kernels": {
                "density_ms": td * 1e3,
                "force_ms": tf * 1e3,
                "force_algorithmic_GBps": b_force / tf / 1e9,
                "density_fp64_frac": n_density * FLOPS_DENSITY / td / FP64_PEAK,
                "force_fp64_frac": n_force * FLOPS_FORCE / tf / FP64_PEAK,
                # the list build's work counters of the counted setup loop
                # (swh_list.h TileStats): candidates loaded, staged, candidate-test
                # steps and list-flush steps (force: zeros, it reuses the lists)
                "density_loop_stats": stats_density,
                "force_loop_stats": stats_force,
            },
            "cpu_baseline": None,
            "ranks": RANKS,
        }
        if halo:
            out["halo_exchange"] = {
                "per_rank": halo,
                "note": "one rho refresh per step between the density and force loops "
                        "(decomp.DeviceHalo: pack, batch_isend_irecv, unpack on the space's "
                        "stream); exchange_ms = HIP events around it, mean over the timed steps"}
        if steady:
            out["steady_state"] = steady
        if breakdown:
            out["step_breakdown"] = breakdown
        if eagle and world == 1 and not args.no_cpu_baseline:
            # SWIFT's own CPU path for clustered boxes: the cell tree split to
            # space_splitsize 400 and the DOSUB recursion
            try:
                threads = cpu_share_threads()
                Hmax = KERNEL_GAMMA * float(local["h"].max())
                cdim = max(4, int(float(P.dim[0]) / (Hmax * 1.0001)))
                cdim -= cdim % 2
                w = run_cpu_worker("hydro_tree", {"parts": np.ascontiguousarray(local).view(np.uint8)},
                                   {"dim": list(P.dim), "max_active_bin": int(P.max_active_bin),
                                    "cdim": cdim, "splitsize": 400, "runs": 1}, threads)
                n = n_density + n_force
                out["cpu_baseline"] = {
                    "value": n / w["seconds_share"], "unit": "interactions/s", "cores": threads,
                    "kind": "port", "host": host_cpu_info(),
                    "pinning": "one thread per physical core, child process without torch",
                    "sample": f"the whole box, density + force loops: float restatement of "
                              f"DOSUB_SELF1/PAIR1 + DOSUB_SELF2/PAIR2 recursing over a {cdim}^3 "
                              f"top grid split to <= 400 particles per cell ({w['cells']} cells, "
                              f"cell_can_recurse_in_{{self,pair}}_hydro_task), leaf "
                              f"DOSELF/DOPAIR sorted loops; 1 run after 1 warm-up "
                              f"({w['seconds_share']:.3f} s per step; tree build "
                              f"{w['seconds_tree_build']:.2f} s untimed)"}
                out["gpu_over_cpu"] = out["value"] / out["cpu_baseline"]["value"]
            except Exception as e:  # report, never fake
                log(f"eagle tree cpu baseline failed: {e}")
        elif world == 1 and not args.no_cpu_baseline:
            # the CPU path times the same loops on the same (prepared) inputs:
            # `local` still holds the converged chain state the GPU started from
            try:
                out["cpu_baseline"] = cpu_baseline(local, P, n_density, n_force, args.cpu_runs)
                # vs the CPU share of one GPU (measured); vs every physical core of
                # the host (projected from the measured per-thread rate)
                out["gpu_over_cpu"] = out["value"] / out["cpu_baseline"]["value"]
                out["gpu_over_cpu_basis"] = (f"cpu_baseline.value: {out['cpu_baseline']['cores']} "
                                             "pinned threads, one GPU's CPU share")
                out["gpu_over_cpu_full_host_projected"] = (
                    out["value"] / out["cpu_baseline"]["full_host_projected"]["value"])
                fh = out["cpu_baseline"].get("full_host") or {}
                if fh.get("value"):
                    out["gpu_over_cpu_full_host_measured"] = out["value"] / fh["value"]
            except Exception as e:  # report, never fake
                log(f"cpu baseline failed: {e}")
            try:
                tuning = (args.cell_factor, args.loop_variant, args.group_size, args.cell_scale,
                          0, args.list_capacity, args.list_skin)
                out["parity"] = parity_vs_cpu(ctx, local, P, tuning,
                                              out["cpu_baseline"]["cores"]
                                              if out["cpu_baseline"] else 16, args.workload)

            except Exception as e:  # report, never fake
                log(f"parity check failed: {e}")
        if raw is not None:
            try:
                out.setdefault("parity", {})["chain_vs_f32"] = chain_vs_f32(
                    raw, chain_gpu, chain, P, args.workload)
            except Exception as e:  # report, never fake
                log(f"chain parity check failed: {e}")
            if not eagle:
                try:
                    out.setdefault("parity", {})["flow_vs_f32"] = flow_vs_f32(ctx)
                except Exception as e:  # report, never fake
                    log(f"flow parity check failed: {e}")
    sp.close()
    ctx.close()
    if rank == 0:
        if (world == 1 and not eagle and strong and not args.no_configs and args.n == 128
                and args.diag_mode == 0):
            # the other BASELINE configs, each its own bench.py run after this
            # process has released its GPU memory (untimed by the headline)
            out["configs"] = other_configs(args)
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
