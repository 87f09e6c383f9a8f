#!/bin/bash
# Parity suites, then the headline bench twice (density / force ms).
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400:t_par:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_physics.py tests/test_gpu_drift.py tests/test_dosub.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
for k in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 30 > gpurun_out/bench$k.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench$k.log').read().strip().splitlines()[-1]); print('ms', round(d['ms_per_step'],4), 'dens', round(d['kernels']['density_ms'],4), 'force', round(d['kernels']['force_ms'],4), 'value', '%.4g' % d['value'])"
done
