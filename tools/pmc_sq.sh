#!/bin/bash
# SQ instruction-mix / stall counters of the tile loop kernels (kernel-trace
# only, one PMC pass per counter set). usage: tools/pmc_sq.sh <variant>...
set -o pipefail
mkdir -p gpurun_out
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for v in "$@"; do
  for p in A B; do
    timeout -s KILL 90 rocprofv3 --pmc ${!p} --kernel-include-regex "tile" -d gpurun_out/sq_v${v}_$p \
      -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 2 --warmup 1 \
      --loop-variant $v > gpurun_out/sq_v${v}_$p.log 2>&1 || exit $?
  done
done
