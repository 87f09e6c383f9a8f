#!/usr/bin/env python3
"""Median duration per kernel of a rocprofv3 kernel_trace.csv, over the last
N dispatches of each kernel (the bench's timed steps come last).
usage: ktrace_median.py <kernel_trace.csv> [last_n]"""
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
by = {}
for r in rows:
    name = re.sub(r"\(.*", "", r["Kernel_Name"])
    name = re.sub(r"rocprim::ROCPRIM_\w+::detail::", "rocprim::", name)[:60]
    by.setdefault(name, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
out = []
for k, v in by.items():
    v.sort()
    d = [x[1] for x in v[-last:]]
    out.append((statistics.median(d) / 1e3, len(v), k))
for med, n, k in sorted(out, reverse=True)[:25]:
    print(f"{k:60s} n {n:5d} median(last) {med:9.1f} us")
