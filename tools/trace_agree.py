"""Agreement of the bench line's event-timed loop with the rocprofv3 kernel
trace of the same command: the mean duration of the last `steps` dispatches
of each loop kernel (the timed steps come last in a --no-steady
--no-breakdown run) against the line's density_ms / force_ms.
usage: python tools/trace_agree.py <trace csv> <bench line json> <steps> [out json]"""
import csv
import json
import statistics
import sys
from collections import defaultdict

trace, line, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
d = json.loads([l for l in open(line) if l.startswith("{")][-1])
by = defaultdict(list)
for r in rows:
    by[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
dens = ["swh::group_prep_kernel", "swh::list_build_kernel", "void swh::density_walk_kernel<double>",
        "void swh::overflow_kernel<0, double>"]
force = ["void swh::walk_kernel<2, double>", "void swh::overflow_kernel<2, double>"]
out = {"kernels_us": {}, "line": {"density_ms": d["kernels"]["density_ms"],
                                  "force_ms": d["kernels"]["force_ms"]}}
for k in dens + force:
    v = by.get(k, [])[-steps:]
    out["kernels_us"][k] = statistics.mean(v) if v else None
out["trace_density_ms"] = sum(out["kernels_us"][k] or 0 for k in dens) * 1e-3
out["trace_force_ms"] = sum(out["kernels_us"][k] or 0 for k in force) * 1e-3
out["note"] = ("the event-timed loops include the launch gaps between their kernels; "
               "the trace sums kernel durations only")
print(json.dumps(out, indent=1))
if len(sys.argv) > 4:
    open(sys.argv[4], "w").write(json.dumps(out, indent=1) + "\n")
