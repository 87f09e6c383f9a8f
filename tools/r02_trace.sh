#!/bin/bash
# kernel-trace stats of one bench configuration. usage: tools/r02_trace.sh <tag> [bench args]
tag="$1"; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_trace" -o run --output-format csv \
  -- python bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@" > "gpurun_out/${tag}_trace.log" 2>&1 || exit $?
python3 tools/kstats.py "gpurun_out/${tag}_trace/run_kernel_stats.csv"
