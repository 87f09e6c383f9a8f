#!/bin/bash
# Failing-test reruns, the pipelined build/walk A/B (SWH_BUILD_CHUNKS), and
# the pipelined path's parity at 128^3.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:t_fix:python -u -m pytest tests/test_gpu_physics.py tests/test_gpu_drift.py -q --timeout 300 --timeout-method thread" \
 "300:t_chunk:SWH_BUILD_CHUNKS=4 python -u -m pytest tests/test_gpu_parity.py -q -k 'headline or box_chain or clustered' --timeout 300 --timeout-method thread" || exit $?
for c in 1 2 4 8 1 4; do
  SWH_BUILD_CHUNKS=$c timeout -k 10 200 python bench.py --no-cpu-baseline --no-breakdown --no-steady --steps 20 > gpurun_out/abc_$c.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/abc_$c.log').read().strip().splitlines()[-1]); print('chunks=$c', round(d['ms_per_step'],4), 'dens', round(d['kernels']['density_ms'],4), 'force', round(d['kernels']['force_ms'],4))"
done
