#!/bin/bash
# Kernel-trace stats of the headline bench and the SQ / TA counters of the
# density loop kernels (one PMC pass each, kernel-trace only).
export TMPDIR=/tmp
tag=${1:-r03i}
out=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${tag}_trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 10 > $out/${tag}_trace.log 2>&1 || exit $?
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
timeout -s KILL 90 rocprofv3 --pmc $A --kernel-include-regex "list_build|walk_kernel" -d $out/${tag}_sq -o run --output-format csv -- python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 2 --warmup 1 > $out/${tag}_sq.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "list_build|walk_kernel" -d $out/${tag}_ta -o run --output-format csv -- python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 2 --warmup 1 > $out/${tag}_ta.log 2>&1 || exit $?
python3 tools/sq_summary.py $out/${tag}_sq $out/${tag}_ta
python3 - <<PY
import csv
rows=list(csv.DictReader(open("$out/${tag}_trace/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-60s calls %5s avg %8.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1e3))
PY
