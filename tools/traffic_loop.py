"""HBM traffic of a hydro workload's density loop from two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE; kernel-trace only): per kernel the median over its
dispatches, FETCH_SIZE x2 (the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md, "HBM"), KiB -> bytes; the density
loop's bytes per launch = the sum over its kernels. The overflow kernels are
taken at the main loops' grid (64 workgroups) only: the ghost's rerun
searches launch the same kernel on larger grids.
usage: python tools/traffic_loop.py <pmc tag> <workload>
  reads gpurun_out/<tag>_pmc_{FETCH_SIZE,WRITE_SIZE}/run_counter_collection.csv,
  writes profiles/traffic_<workload>.json (traffic_density.json for sedov; bench.py
  load_traffic)."""
import collections
import csv
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def measured_commit():
    """The commit whose kernels the PMC passes ran (the tree gpurun shipped
    is HEAD when this runs right after the call; '+dirty' if csrc/ differs)."""
    import subprocess
    try:
        c = subprocess.run(["git", "-C", str(ROOT), "rev-parse", "--short", "HEAD"],
                           capture_output=True, text=True).stdout.strip()
        d = subprocess.run(["git", "-C", str(ROOT), "status", "--porcelain", "--",
                            "swift_subtask_dev_amd/csrc"], capture_output=True, text=True).stdout
        return c + ("+dirty" if d.strip() else "")
    except OSError:
        return None

DENSITY = ["swh::posf_kernel", "swh::group_box_kernel", "swh::cell_reach_kernel", "swh::group_prep_kernel", "swh::list_build_kernel",
           "void swh::density_walk_kernel<double>", "void swh::overflow_kernel<0, double>"]
MAIN_OVF_GRID = 64 * 256

tag, workload = sys.argv[1:3]
med = collections.defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = ROOT / "gpurun_out" / f"{tag}_pmc_{c}" / "run_counter_collection.csv"
    per = collections.defaultdict(float)  # (kernel, dispatch) -> value summed over rows
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "overflow_kernel" in k and int(r["Grid_Size"]) != MAIN_OVF_GRID:
            continue
        per[(k, r["Dispatch_Id"])] += float(r["Counter_Value"])
    by = collections.defaultdict(list)
    for (k, _), v in per.items():
        by[k].append(v)
    for k, v in by.items():
        med[k][c] = statistics.median(v)
kern = {}
for k, m in sorted(med.items()):
    rd = 2.0 * m.get("FETCH_SIZE", 0.0) * 1024
    wr = m.get("WRITE_SIZE", 0.0) * 1024
    kern[k] = {"read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr}
dens = [k for k in DENSITY if k in kern]
out = {"commit": measured_commit(), "source": f"profiles/{tag} PMC passes (rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE, "
                 "kernel-trace only; FETCH_SIZE x2 gfx950 correction; median over dispatches; "
                 "overflow kernels at the main loops' grid)",
       "kernels": kern, "density_kernels": dens,
       "bytes_per_launch": sum(kern[k]["bytes_per_launch"] for k in dens)}
# bench.py load_traffic: the Sedov headline reads traffic_density.json
name = "traffic_density.json" if workload == "sedov" else f"traffic_{workload}.json"
(ROOT / "profiles" / name).write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps({k: round(v["bytes_per_launch"] / 1e6, 1) for k, v in kern.items()}),
      "density loop MB:", round(out["bytes_per_launch"] / 1e6, 1))
