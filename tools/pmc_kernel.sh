#!/bin/bash
# SQ / fp64 instruction-mix / LDS / TA counters of the kernels matching a
# regex over a bench.py run: one PMC pass per counter set (each within the
# per-block limits: <= 8 SQ, <= 2 TA, <= 2 GRBM), kernel-trace only, no
# trace domains.
# usage: tools/pmc_kernel.sh <tag> <kernel regex> <bench args...>
#   -> gpurun_out/<tag>_{A,B,C,D}/ ; python tools/sq_json.py gpurun_out/<tag> > <json>
tag="$1"; regex="$2"; shift 2
set -o pipefail
mkdir -p gpurun_out
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
B="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_CVT"
D="TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE"
for p in A B C D; do
  timeout -s KILL 120 rocprofv3 --pmc ${!p} --kernel-include-regex "$regex" -d gpurun_out/${tag}_$p \
    -o run --output-format csv -- python bench.py --no-configs --no-cpu-baseline "$@" \
    > gpurun_out/${tag}_$p.log 2>&1 || exit $?
done
python tools/sq_json.py gpurun_out/${tag} > gpurun_out/${tag}_sq.json
