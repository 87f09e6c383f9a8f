#!/bin/bash
# Two i-groups per list-build wave (group_size 32, shared staging) against
# one: parity of the group-32 cases, then the headline bench alternating.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:t_g32:python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k 32" || exit $?
one() {  # tag, env, group size
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 30 --group-size $3 > gpurun_out/bench_$1.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bench_$1.log').read().strip().splitlines()[-1]); k=d['kernels']; print('$1', 'ms', round(d['ms_per_step'],4), 'dens', round(k['density_ms'],4), 'force', round(k['force_ms'],4), 'value', '%.4g' % d['value'], k['density_loop_stats'])"
}
for k in 1 2; do
one g16_$k X=1 16
one g32_$k X=1 32
one g32wpe4_$k SWH_LIB_PATH=swift_subtask_dev_amd/_exp/wpe4.so 32
one g32r192_$k SWH_LIB_PATH=swift_subtask_dev_amd/_exp/rh192.so 32
done
