"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) per kernel:
mean counter values per dispatch and derived per-wave figures."""
import collections
import csv
import sys
from pathlib import Path

root = Path(sys.argv[1])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(root.glob("*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(f"== {k}")
    w = m.get("SQ_WAVES", 0)
    for c in sorted(m):
        extra = f"  ({m[c] / w:.4g}/wave)" if w and c.startswith("SQ_") and c != "SQ_WAVES" else ""
        print(f"   {c:24s} {m[c]:.4g}{extra}")
    if "FETCH_SIZE" in m:
        print(f"   HBM read (x2 gfx950 corr.) {2 * m['FETCH_SIZE'] * 1024 / 1e9:.3f} GB/dispatch")
    if "WRITE_SIZE" in m:
        print(f"   HBM write {m['WRITE_SIZE'] * 1024 / 1e9:.3f} GB/dispatch")
