#!/bin/bash
# Round-3 closing set (final): GPU suite + smoke, headline profile (bench line with CPU
# baseline, kernel trace, FETCH/WRITE PMC), SQ and TA counters of the density
# loop kernels, and the eagle / grav 256^3 / cosmo lines.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" || exit $?
KREGEX="list_build|walk_kernel|overflow_kernel|posf_kernel|list_prep|cell_reach|init_kernel|reset_acc" \
  tools/profile_round.sh r03s || exit $?
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
timeout -s KILL 90 rocprofv3 --pmc $A --kernel-include-regex "list_build|walk_kernel" -d gpurun_out/r03s_sq -o run --output-format csv -- python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 3 --warmup 1 > gpurun_out/r03s_sq.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "list_build|walk_kernel" -d gpurun_out/r03s_ta -o run --output-format csv -- python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 3 --warmup 1 > gpurun_out/r03s_ta.log 2>&1 || exit $?
tools/gpu_steps.sh \
 "400:r03s_eagle:python bench.py --workload eagle --steps 10 --warmup 3" \
 "400:r03s_grav:python bench.py --workload grav --n 256 --steps 3 --warmup 1" \
 "300:r03s_cosmo:python bench.py --workload cosmo --steps 10 --warmup 3"
