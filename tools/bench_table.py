#!/usr/bin/env python3
"""Print config + kernel times of the bench JSON line in gpurun_out/<name>.log."""
import json
import sys

for name in sys.argv[1:]:
    try:
        lines = [x for x in open(f"gpurun_out/{name}.log") if x.startswith("{")]
        d = json.loads(lines[-1])
        c, k = d["config"], d["kernels"]
        print(f"{name:8s} density {k['density_ms']:.3f} ms force {k['force_ms']:.3f} ms "
              f"step {d['ms_per_step']:.3f} ms value {d['value']:.3g} frac {d['roofline']['frac']:.3f} "
              f"list {c.get('list_entries')} ovf {c.get('list_overflow')}")
    except Exception as e:  # noqa: BLE001
        print(name, "n/a", e)
