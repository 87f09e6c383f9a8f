#!/bin/bash
# quick A/B: list-path parity on small boxes, then the headline bench (no CPU leg)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:t_box:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'box'" \
 "200:b0:python -u bench.py --no-cpu-baseline --no-breakdown $BENCH_ARGS"
python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/b0.log') if l.startswith('{')][-1]); print('b0', d['value'], d['kernels']['density_ms'], d['kernels']['force_ms'])"
