"""HBM traffic of one workload's roofline kernel from two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE; kernel-trace only), per launch, median over its
dispatches: FETCH_SIZE x2 (the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md, "HBM"), KiB -> bytes.
usage: python tools/traffic_json.py <tag> <workload> <kernel substring>
  reads gpurun_out/<tag>_pmc_{FETCH_SIZE,WRITE_SIZE}/run_counter_collection.csv,
  writes profiles/traffic_<workload>.json (bench.py load_traffic)."""
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

tag, workload, sub = sys.argv[1:4]
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = ROOT / "gpurun_out" / f"{tag}_pmc_{c}" / "run_counter_collection.csv"
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if sub in r["Kernel_Name"]]
    if not v:
        sys.exit(f"no {sub} dispatches in {f}")
    vals[c] = statistics.median(v)
rd = 2.0 * vals["FETCH_SIZE"] * 1024
wr = vals["WRITE_SIZE"] * 1024
out = {"commit": measured_commit(), "source": f"profiles/{tag} PMC passes (rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE, "
                 "kernel-trace only; FETCH_SIZE x2 gfx950 correction; median over dispatches)",
       "kernel": sub, "read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr}
(ROOT / "profiles" / f"traffic_{workload}.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out, indent=1))
