#!/bin/bash
# Group walk: counters, PMC of the walks, chunk-size A/B.
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 20"
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'ms', round(d['ms_per_step'],4), 'dens', round(d['kernels']['density_ms'],4), 'force', round(d['kernels']['force_ms'],4), 'fstats', d['kernels']['force_loop_stats'])" $1 $2; }
timeout -k 10 200 $B > gpurun_out/b0.log 2>&1 && summ gpurun_out/b0.log base || exit $?
for v in gw_f128 gw_d64; do
  SWH_LIB_PATH=swift_subtask_dev_amd/_exp/$v.so timeout -k 10 200 $B > gpurun_out/b_$v.log 2>&1 && summ gpurun_out/b_$v.log $v || exit $?
done
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
timeout -s KILL 90 rocprofv3 --pmc $A --kernel-include-regex "group_walk|list_build" -d gpurun_out/pmcA -o run --output-format csv -- python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 2 --warmup 1 > gpurun_out/pmcA.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "group_walk|list_build" -d gpurun_out/pmcB -o run --output-format csv -- python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 2 --warmup 1 > gpurun_out/pmcB.log 2>&1 || exit $?
python3 tools/sq_summary.py gpurun_out/pmcA gpurun_out/pmcB > gpurun_out/pmc_sum.txt 2>&1; tail -60 gpurun_out/pmc_sum.txt
