"""Average SQ PMC counters per tile kernel from tools/pmc_sq.sh output.

usage: python tools/sq_summary.py gpurun_out/sq_v4_A gpurun_out/sq_v4_B ...
"""
import collections
import csv
import sys


def main(dirs):
    for d in dirs:
        rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in rows:
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in agg.items():
            vals = {c: "%.4g" % (sum(x) / len(x)) for c, x in sorted(cs.items())}
            print(d.rstrip("/").split("/")[-1], k, vals)


if __name__ == "__main__":
    main(sys.argv[1:])
