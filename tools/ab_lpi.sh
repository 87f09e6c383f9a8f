#!/bin/bash
# walk lanes-per-i A/B: the default library, then var_so/ builds with 2 and 8
export TMPDIR=/tmp
cp swift_subtask_dev_amd/libswifthip.so /tmp/base.so
tools/gpu_steps.sh "200:l4:python -u bench.py --no-cpu-baseline --no-breakdown"
for L in 2 8; do
  cp var_so/libswifthip_lpi$L.so swift_subtask_dev_amd/libswifthip.so
  tools/gpu_steps.sh "200:l$L:python -u bench.py --no-cpu-baseline --no-breakdown" || break
done
cp /tmp/base.so swift_subtask_dev_amd/libswifthip.so
for f in l4 l2 l8; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print('$f', d['value'], d['kernels']['density_ms'], d['kernels']['force_ms'])"; done
