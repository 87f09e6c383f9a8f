#!/bin/bash
# Round profile: full bench line (with CPU baseline), rocprofv3 kernel-trace
# stats of the same bench command, and HBM traffic of the loop kernels from
# PMC (FETCH_SIZE and WRITE_SIZE in separate passes, kernel-trace only).
# usage: tools/profile_round.sh <tag>     -> gpurun_out/<tag>_*
tag="$1"
KREGEX="${KREGEX:-list_build|walk_kernel|overflow_kernel|group_prep|cell_reach|init_kernel|reset_kernel}"
set -o pipefail
out=gpurun_out
timeout -k 10 300 python bench.py --no-configs > "$out/${tag}_bench.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/${tag}_trace" -o run --output-format csv \
  -- python bench.py --no-configs --no-cpu-baseline > "$out/${tag}_trace.log" 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex "$KREGEX" -d "$out/${tag}_pmc_$c" \
    -o run --output-format csv -- python bench.py --no-configs --no-cpu-baseline --steps 5 --warmup 1 \
    --no-steady --no-breakdown \
    > "$out/${tag}_pmc_$c.log" 2>&1 || exit $?
done
echo "profile $tag done"
