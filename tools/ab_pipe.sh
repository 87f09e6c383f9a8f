#!/bin/bash
# density walk software pipeline: parity (all GPU tests) then the bench
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "600:t_all:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200:bp:python -u bench.py --no-cpu-baseline --no-breakdown"
python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bp.log') if l.startswith('{')][-1]); print('bp', d['value'], d['kernels']['density_ms'], d['kernels']['force_ms'], 'reuse', d['step_lists_reused']['density_ms'], d['step_lists_reused']['ms_per_step'], d['step_lists_reused']['density_roofline_frac'])"
