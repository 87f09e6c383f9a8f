#!/bin/bash
# Fused build + density walk: parity, then A/B against the separate walk.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:t_fix3:python -u -m pytest tests/test_gpu_physics.py tests/test_gpu_drift.py -q --timeout 300 --timeout-method thread" \
 "300:t_fused:python -u -m pytest tests/test_gpu_parity.py -q -k 'headline or box_ or clustered or non_periodic or active' --timeout 300 --timeout-method thread" || exit $?
for f in 0 1 0 1; do
  SWH_FUSED_DENSITY=$f timeout -k 10 200 python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 20 > gpurun_out/abf_$f.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/abf_$f.log').read().strip().splitlines()[-1]); print('fused=$f', round(d['ms_per_step'],4), 'dens', round(d['kernels']['density_ms'],4), 'force', round(d['kernels']['force_ms'],4))"
done
