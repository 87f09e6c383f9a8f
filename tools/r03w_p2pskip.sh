#!/bin/bash
# P2P: skip i-slots no lane of the wave holds (SWH_P2P_SKIP) against the
# previous kernel: gravity parity suites, then grav 256^3 and cosmo A/B.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400:t_grav:python -u -m pytest tests/test_gpu_grav_tasks.py tests/test_gpu_tree.py tests/test_gpu_mpole.py tests/test_gpu_parity.py -k 'grav or tree or mpole or Potential' -x -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider" || exit $?
one() {  # tag, env, workload args
  env $2 timeout -k 10 300 python bench.py --no-cpu-baseline $3 > gpurun_out/bench_$1.log 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_$1.log') if l.startswith('{')][-1]); print('$1', 'ms', round(d['ms_per_step'],3), 'value', '%.4g' % d['value'])"
}
for k in 1 2; do
one skip_$k X=1 "--workload grav --n 256 --steps 3 --warmup 1"
one noskip_$k SWH_LIB_PATH=swift_subtask_dev_amd/_exp/noskip.so "--workload grav --n 256 --steps 3 --warmup 1"
done
one cskip X=1 "--workload cosmo --steps 10 --warmup 3"
one cnoskip SWH_LIB_PATH=swift_subtask_dev_amd/_exp/noskip.so "--workload cosmo --steps 10 --warmup 3"
