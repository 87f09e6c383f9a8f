#!/bin/bash
# i-group A/B: octree leaves (default) vs fixed 16-particle chunks of the sorted order
export TMPDIR=/tmp
tools/gpu_steps.sh "200:g0:python -u bench.py --no-cpu-baseline --no-breakdown" \
 "200:g1:SWH_GROUP_CHUNK=1 python -u bench.py --no-cpu-baseline --no-breakdown" \
 "200:t1:SWH_GROUP_CHUNK=1 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k box"
for f in g0 g1; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print('$f', d['value'], d['kernels']['density_ms'], d['kernels']['force_ms'], d['config']['i_groups'], d['kernels']['density_loop_stats'])"; done
tail -1 gpurun_out/t1.log
