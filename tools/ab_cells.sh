#!/bin/bash
# list build A/B over the neighbour-grid cell size (cells per H_max)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "200:c1:python -u bench.py --no-cpu-baseline --no-breakdown" \
 "200:c15:python -u bench.py --no-cpu-baseline --no-breakdown --cell-scale 1.5" \
 "200:c2:python -u bench.py --no-cpu-baseline --no-breakdown --cell-factor 2" \
 "200:c3:python -u bench.py --no-cpu-baseline --no-breakdown --cell-factor 3"
for f in c1 c15 c2 c3; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print('$f', d['value'], d['kernels']['density_ms'], d['kernels']['force_ms'], d['kernels']['density_loop_stats'])"; done
