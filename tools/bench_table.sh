#!/bin/bash
# Print config + kernel times of bench JSON lines in gpurun_out/<name>.log
for f in "$@"; do
python3 - "$f" <<'PY'
import json, sys
name = sys.argv[1]
try:
    l = [x for x in open(f"gpurun_out/{name}.log") if x.startswith("{")]
    d = json.loads(l[-1])
    c = d["config"]
    print(f"{name:10s} groups {c.get('i_groups')} cdim {c.get('grid_cdim')} density {d['kernels']['density_ms']:.3f} ms "
          f"force {d['kernels']['force_ms']:.3f} ms value {d['value']:.3g} frac {d['roofline']['frac']:.3f}")
except Exception as e:
    print(name, "n/a", e)
PY
done
