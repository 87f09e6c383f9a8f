#!/bin/bash
# Density-walk bound (profiling only): per-kernel averages under diag modes
# 0 (full), 3 (walk loads without the math), 4 (walk math on fixed-j loads).
export TMPDIR=/tmp
for d in 0 3 4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/dw_$d -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 10 --warmup 2 --diag-mode $d > gpurun_out/dw_$d.log 2>&1 || exit $?
  f=$(find gpurun_out/dw_$d -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'walk_kernel' in n or 'list_build' in n: print('diag=$d', n[:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
done
