"""Whole-step kernel profile: drift + rebuild + SPHENIX chain on the bench's
128^3 Sedov box (run under rocprofv3 --kernel-trace --stats)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from swift_subtask_dev_amd import abi, ics, lib

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
skin = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
parts = ics.sedov_slabs(n, 1)
P = abi.default_hydro_params((1.0, 1.0, 1.0), True)
P.max_active_bin = 1
ctx = lib.Context(0, "f64")
sp = lib.HydroSpace(ctx)
sp.set_tuning(1, 0, 0, list_skin=skin)
stream = torch.cuda.Stream()
sp.set_stream(stream.cuda_stream)
sp.upload(parts)
sp.rebuild(P)
sp.hydro_step(P)
g = abi.copy_parts(parts)
sp.download(g, abi.FIELDS_ALL)
rng = np.random.Generator(np.random.PCG64(17))
xp = abi.new_xparts(len(parts))
xp["v_full"] = rng.normal(0, 0.577, (len(parts), 3)).astype(np.float32)
sp.upload_xparts(xp)
h = float(np.median(g["h"]))
dt = 0.1 * h / float(np.abs(xp["v_full"]).max() * 1.733)
dt_cfl = min(dt, 0.1 * float(np.min(g["h"] / np.maximum(g["v_sig"], 1e-30))))
D = abi.DriftParams(dt, dt_cfl, dt_cfl, dt_cfl, 0.0)
names = ["drift", "rebuild", "density", "ghost", "gradient", "extra_ghost", "force"]
for k in range(steps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(8)]
    ev[0].record(stream)
    sp.drift(D, P)
    ev[1].record(stream)
    sp.rebuild(P)
    ev[2].record(stream)
    sp.init_parts(P)
    sp.density(P, count=False)
    ev[3].record(stream)
    it, _ = sp.ghost(P)
    ev[4].record(stream)
    sp.gradient(P, count=False)
    ev[5].record(stream)
    sp.extra_ghost(P)
    ev[6].record(stream)
    sp.force(P, count=False)
    sp.end_force(P)
    ev[7].record(stream)
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) for i in range(7)]
    print(f"step {k}: ghost its {it} list_valid {sp.info()['list_valid']} " +
          " ".join(f"{nm} {x:.3f}" for nm, x in zip(names, t)) + f" total {sum(t):.3f} ms",
          flush=True)
