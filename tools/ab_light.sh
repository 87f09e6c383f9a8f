#!/bin/bash
# density walk A/B: particle data two entries ahead (default) vs loaded at the entry (6 waves/SIMD)
export TMPDIR=/tmp
cp swift_subtask_dev_amd/libswifthip.so /tmp/base.so
tools/gpu_steps.sh "200:q2:python -u bench.py --no-cpu-baseline --no-breakdown"
cp var_so/libswifthip_lp0.so swift_subtask_dev_amd/libswifthip.so
tools/gpu_steps.sh "200:q0:python -u bench.py --no-cpu-baseline --no-breakdown" \
 "300:tq:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'box or 128 or reuse'"
cp /tmp/base.so swift_subtask_dev_amd/libswifthip.so
for f in q2 q0; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print('$f', d['value'], d['kernels']['density_ms'], d['kernels']['force_ms'], 'reuse', d['step_lists_reused']['density_ms'], d['step_lists_reused']['ms_per_step'])"; done
tail -1 gpurun_out/tq.log
