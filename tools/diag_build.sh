#!/bin/bash
# List-build time split by diag mode (profiling only, results invalid):
# 0 = build + walk, 1 = build stages candidates only (no tests), 2 = build
# tests but writes no entries. density_ms of each line.
export TMPDIR=/tmp
for d in 0 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-breakdown --steps 20 --diag-mode $d > gpurun_out/diag_$d.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/diag_$d.log').read().strip().splitlines()[-1]); print('diag=$d', 'density_ms', d['kernels']['density_ms'], 'stats', d['kernels']['density_loop_stats'])"
done
