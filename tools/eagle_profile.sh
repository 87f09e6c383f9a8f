#!/bin/bash
# EAGLE_6 stand-in profile beside the Sedov headline (verdict r04 item 6):
# bench lines, kernel-trace stats, PMC traffic (FETCH_SIZE, WRITE_SIZE in
# separate passes) and SQ counter sets of the loop kernels, kernel-trace only.
# usage: tools/eagle_profile.sh <tag>   -> gpurun_out/<tag>_{eagle,sedov}_*
tag="$1"
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out
K="list_build|walk_kernel|overflow_kernel|posf_kernel|group_box|group_prep|init_kernel|reset_acc"
for w in eagle sedov; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-steady --no-breakdown \
    > "$out/${tag}_${w}_bench.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/${tag}_${w}_trace" -o run --output-format csv \
    -- python bench.py --workload $w --no-cpu-baseline --no-steady --no-breakdown --steps 5 --warmup 1 \
    > "$out/${tag}_${w}_trace.log" 2>&1 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "$K" -d "$out/${tag}_${w}_pmc_$c" \
      -o run --output-format csv -- python bench.py --workload $w --no-cpu-baseline --steps 3 --warmup 1 \
      --no-steady --no-breakdown > "$out/${tag}_${w}_pmc_$c.log" 2>&1 || exit $?
  done
  bash tools/pmc_kernel.sh "${tag}_${w}_sq" "$K" --workload $w --steps 3 --warmup 1 --no-steady --no-breakdown || exit $?
  echo "$w done"
done
