#!/bin/bash
# List-build VALU/SALU/LDS instruction split by diag mode (1 = staging only,
# 2 = staging + tests, 0 = full) and the walk, one PMC pass per mode.
export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
for d in 1 2 0; do
  timeout -s KILL 90 rocprofv3 --pmc $A --kernel-include-regex "list_build|walk_kernel" -d gpurun_out/pd$d -o run --output-format csv -- python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 2 --warmup 1 --diag-mode $d > gpurun_out/pd$d.log 2>&1 || exit $?
done
python3 tools/sq_summary.py gpurun_out/pd1 gpurun_out/pd2 gpurun_out/pd0
