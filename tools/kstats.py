#!/usr/bin/env python3
"""Short table of a rocprofv3 kernel_stats.csv: calls, mean and total ms per kernel."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 14]:
    name = re.sub(r"\(.*", "", r["Name"])
    name = re.sub(r"rocprim::ROCPRIM_\w+::detail::", "rocprim::", name)[:70]
    print(f"{name:70s} calls {int(r['Calls']):4d} mean {float(r['AverageNs']) / 1e6:8.4f} ms "
          f"total {float(r['TotalDurationNs']) / 1e6:8.3f} ms")
