#!/bin/bash
# per-config lines (SURVEY 8d / north_star): Sedov 64^3..256^3 sweep, EAGLE_6
# stand-in, gravity 256^3 P2P
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "200:sw64:python -u bench.py --n 64 --no-cpu-baseline --no-breakdown" \
 "200:sw128:python -u bench.py --n 128 --no-cpu-baseline --no-breakdown" \
 "300:sw256:python -u bench.py --n 256 --no-cpu-baseline --no-breakdown --steps 5" \
 "300:eagle:python -u bench.py --workload eagle --no-cpu-baseline" \
 "400:grav:python -u bench.py --workload grav --n 256 --steps 5 --warmup 1"
for f in sw64 sw128 sw256 eagle grav; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d.get('kernels',{}).get('density_ms'), d.get('kernels',{}).get('force_ms'), d['roofline']['frac'])"; done
