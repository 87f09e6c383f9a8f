#!/bin/bash
# Bench A/B only: default vs variant(s).
export TMPDIR=/tmp
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'ms', round(d['ms_per_step'],4), 'dens', round(d['kernels']['density_ms'],4), 'force', round(d['kernels']['force_ms'],4), 'value', '%.4g' % d['value'])" $1 $2; }
B="python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 30"
for rep in 1 2; do
  timeout -k 10 200 $B > gpurun_out/b_def$rep.log 2>&1 && summ gpurun_out/b_def$rep.log default || exit $?
  for v in "$@"; do
    SWH_LIB_PATH=swift_subtask_dev_amd/_exp/$v.so timeout -k 10 200 $B > gpurun_out/b_$v$rep.log 2>&1 && summ gpurun_out/b_$v$rep.log $v || exit $?
  done
done
