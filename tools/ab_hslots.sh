#!/bin/bash
# gradient/force walk A/B: record at its entry (default) vs a two-slot pipeline (152 VGPRs, 3 waves)
export TMPDIR=/tmp
cp swift_subtask_dev_amd/libswifthip.so /tmp/base.so
tools/gpu_steps.sh "200:h0:python -u bench.py --no-cpu-baseline"
cp var_so/libswifthip_hs2.so swift_subtask_dev_amd/libswifthip.so
tools/gpu_steps.sh "200:h2:python -u bench.py --no-cpu-baseline" \
 "300:th:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'box or 128'"
cp /tmp/base.so swift_subtask_dev_amd/libswifthip.so
for f in h0 h2; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); b=d['step_breakdown']['rebuild_every_step']; print('$f', d['value'], d['kernels']['density_ms'], d['kernels']['force_ms'], 'grad', b['gradient_ms'])"; done
tail -1 gpurun_out/th.log
