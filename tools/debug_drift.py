"""Drift debugging on the bench's state (prints h/x/dx stats after a drift)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from swift_subtask_dev_amd import abi, ics, lib

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
parts = ics.sedov_slabs(n, 1)
P = abi.default_hydro_params((1.0, 1.0, 1.0), True)
P.max_active_bin = 1
ctx = lib.Context(0, "f64")
sp = lib.HydroSpace(ctx)
stream = torch.cuda.Stream()
sp.set_stream(stream.cuda_stream)
sp.upload(parts)
sp.rebuild(P)
sp.hydro_step(P)
g = abi.copy_parts(parts)
sp.download(g, abi.FIELDS_ALL)
print("after chain: h", g["h"].min(), g["h"].max(), "h_dt", np.abs(g["h_dt"]).max(),
      "u", g["u"].min(), g["u"].max(), "u_dt", g["u_dt"].min(), g["u_dt"].max(), flush=True)
print("info", sp.info(), flush=True)
rng = np.random.Generator(np.random.PCG64(17))
xp = abi.new_xparts(len(parts))
xp["v_full"] = rng.normal(0, 0.577, (len(parts), 3)).astype(np.float32)
sp.upload_xparts(xp)
h = float(np.median(g["h"]))
dt = 0.1 * h / float(np.abs(xp["v_full"]).max() * 1.733)
print("dt", dt, flush=True)
D = abi.DriftParams(dt, dt, dt, dt, 0.0)
try:
    sp.drift(D, P)
except Exception as e:
    print("drift error", e, flush=True)
sp.download(g, abi.FIELDS_ALL)
print("after drift: h", g["h"].min(), g["h"].max(), "x", g["x"].min(), g["x"].max(),
      "nan h", np.isnan(g["h"]).sum(), flush=True)
print("info", sp.info(), flush=True)
