"""Debug: per-step state of the steady-state loop on a small clustered box
(the EAGLE stand-in's steady state reported zero interactions after step 1)."""
import numpy as np
import torch
from swift_subtask_dev_amd import abi, ics, lib

ctx = lib.Context(0)
parts = ics.clustered_box(40, n_clumps=8, per_clump=4000, seed=6)
P = abi.default_hydro_params((1.0, 1.0, 1.0), True)
P.max_active_bin = 1
sp = lib.HydroSpace(ctx)
sp.upload(parts)
sp.rebuild(P)
sp.hydro_step(P)
sp.download(parts, abi.FIELDS_ALL)
sp.close()
print("tb", np.unique(parts["time_bin"], return_counts=True), "h", parts["h"].min(), parts["h"].max())
sp = lib.HydroSpace(ctx)
sp.set_tuning(list_skin=0.01)
sp.upload(parts)
sp.rebuild(P)
n = len(parts)
rng = np.random.Generator(np.random.PCG64(23))
xp = abi.new_xparts(n)
xp["v_full"] = rng.normal(0.0, 0.577, (n, 3)).astype(np.float32)
vmax = float(np.sqrt((xp["v_full"].astype(np.float64) ** 2).sum(axis=1)).max())
dt = 0.05 * float(parts["h"].min()) / vmax
sp.upload_xparts(xp)
D = abi.DriftParams(dt, 0.0, 0.0, 0.0, 0.0)
for k in range(4):
    sp.reset_acceleration(P)
    sp.drift(D, P)
    sp.init_parts(P)
    r = sp.density(P, count=True)
    q = sp.force(P, count=True)
    out = abi.copy_parts(parts)
    sp.download(out, abi.FIELDS_ALL)
    x = out["x"].astype(np.float64)
    print(k, "density", r, "force", q, "nan x", int(np.isnan(x).sum()), "nan h", int(np.isnan(out["h"]).sum()),
          "h", float(np.nanmin(out["h"])), float(np.nanmax(out["h"])), "tb", np.unique(out["time_bin"])[:5],
          "info", {kk: sp.info()[kk] for kk in ("list_valid", "dx_max", "list_builds", "list_overflow")})
