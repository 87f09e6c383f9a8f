"""Copy a round's profile outputs from gpurun_out/ into profiles/ (tracked):
the bench JSON line, the rocprofv3 kernel-trace stats, and the per-launch
HBM traffic of the tile loop kernels from PMC FETCH_SIZE / WRITE_SIZE
(gfx950: FETCH_SIZE counts half the bytes of wide reads -> x2, per
/opt/skills/guides/MI355X_MICROARCH.md "HBM"; the units are KiB).
usage: python tools/make_profiles.py <tag>"""
import csv
import json
import shutil
import statistics
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
tag = sys.argv[1]
src = ROOT / "gpurun_out"
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)

lines = [l for l in open(src / f"{tag}_bench.log") if l.startswith("{")]
bench = json.loads(lines[-1])
(dst / f"{tag}_bench.json").write_text(json.dumps(bench, indent=1) + "\n")

stats = src / f"{tag}_trace" / "run_kernel_stats.csv"
shutil.copy(stats, dst / f"{tag}_kernel_stats.csv")
trace_bench = [l for l in open(src / f"{tag}_trace.log") if l.startswith("{")]
if trace_bench:
    (dst / f"{tag}_trace_bench.json").write_text(trace_bench[-1])

per = defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = src / f"{tag}_pmc_{c}" / "run_counter_collection.csv"
    vals = defaultdict(list)
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in vals.items():
        per[k][c] = statistics.median(v)
traffic = {}
for k, v in per.items():
    rd = 2.0 * v.get("FETCH_SIZE", 0.0) * 1024
    wr = v.get("WRITE_SIZE", 0.0) * 1024
    traffic[k] = {"read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr}
out = {"source": f"profiles/{tag} PMC passes (rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE, "
                 "kernel-trace only; FETCH_SIZE x2 gfx950 correction; median over dispatches)",
       "kernels": traffic}
# one density loop of the list path = the kernels it launches: positions
# staging, list prep + build, the walk and the overflow search
DENSITY_LIST = ("group_prep_kernel", "cell_reach_kernel", "list_build_kernel",
                "walk_kernel<0, double>", "density_walk_kernel<double>",
                "overflow_kernel<0, double>")
parts = {k: v for k, v in traffic.items() if any(k.endswith(d) or d in k for d in DENSITY_LIST)}
if parts:
    out["density_kernels"] = sorted(parts)
    out["bytes_per_launch"] = sum(v["bytes_per_launch"] for v in parts.values())
(dst / f"{tag}_traffic.json").write_text(json.dumps(out, indent=1) + "\n")
(dst / "traffic_density.json").write_text(json.dumps(out, indent=1) + "\n")
dens = [k for k in traffic if "list_build_kernel" in k]

rows = list(csv.DictReader(open(stats)))
print("bench:", bench["value"], bench["kernels"])
for r in rows[:6]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4} avg {float(r["AverageNs"]) / 1e6:.4f} ms')
print(json.dumps(out, indent=1))

# per-dispatch durations of the density kernel from the kernel trace: the
# first dispatches belong to bench.py's untimed setup (full chain + counted
# launch, which also pays the first scratch/page set-up); the last `steps`
# are the timed region, whose mean is what bench.py's HIP events measure
kt = src / f"{tag}_trace" / "run_kernel_trace.csv"
if kt.exists() and dens:
    name = dens[0]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
         for r in csv.DictReader(open(kt)) if r["Kernel_Name"].split("(")[0] == name]
    tb = json.loads(trace_bench[-1]) if trace_bench else {"steps": 10, "warmup": 3}
    steps, warmup = tb["steps"], tb.get("warmup", 3)
    # bench.py's order: the setup chain, then ONE counted density loop (its
    # build counts entries with atomics: the second launch many times the
    # median), then `warmup` untimed and `steps` timed steps; the list-reuse
    # and breakdown sections come after and are not the headline
    med = statistics.median(d)
    slow = [k for k, x in enumerate(d) if x > 4 * med]
    start = (slow[1] + 1 if len(slow) > 1 else 0) + warmup
    timed = d[start:start + steps]
    (dst / f"{tag}_density_dispatches.json").write_text(json.dumps({
        "kernel": name, "dispatch_ms": d, "timed_dispatches": len(timed), "timed_first_index": start,
        "timed_mean_ms": sum(timed) / len(timed), "all_mean_ms": sum(d) / len(d)}, indent=1) + "\n")
