#!/bin/bash
# P2P j-loop unroll A/B on the 256^3 config-4 box: default, var_so/ u2 and u4
export TMPDIR=/tmp
cp swift_subtask_dev_amd/libswifthip.so /tmp/base.so
tools/gpu_steps.sh "300:u1:python -u bench.py --workload grav --n 256 --steps 4 --warmup 1"
for U in 2 4; do
  cp var_so/libswifthip_u$U.so swift_subtask_dev_amd/libswifthip.so
  tools/gpu_steps.sh "300:u$U:python -u bench.py --workload grav --n 256 --steps 4 --warmup 1" || break
done
cp /tmp/base.so swift_subtask_dev_amd/libswifthip.so
for f in u1 u2 u4; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
