#!/bin/bash
# gradient/force walk A/B: data one entry ahead (default) vs loaded at the entry
export TMPDIR=/tmp
cp swift_subtask_dev_amd/libswifthip.so /tmp/base.so
tools/gpu_steps.sh "200:p1:python -u bench.py --no-cpu-baseline"
cp var_so/libswifthip_np.so swift_subtask_dev_amd/libswifthip.so
tools/gpu_steps.sh "200:p0:python -u bench.py --no-cpu-baseline" \
 "300:t0:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'box or 128'"
cp /tmp/base.so swift_subtask_dev_amd/libswifthip.so
for f in p1 p0; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); b=d['step_breakdown']['rebuild_every_step']; print('$f', d['value'], d['kernels']['density_ms'], d['kernels']['force_ms'], 'grad', b['gradient_ms'], 'reuse', d['step_lists_reused']['ms_per_step'])"; done
tail -1 gpurun_out/t0.log
