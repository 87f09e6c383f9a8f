#!/bin/bash
# Group walk (U lists): parity suites, then the headline line.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400:t_par:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_physics.py tests/test_gpu_drift.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "300:bench:python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 20" || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print('ms', round(d['ms_per_step'],4), 'dens', round(d['kernels']['density_ms'],4), 'force', round(d['kernels']['force_ms'],4), 'value', d['value'])"
