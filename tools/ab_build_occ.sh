#!/bin/bash
# list-build occupancy A/B: LDS region / hit cap / staging depth / waves per SIMD
export TMPDIR=/tmp
args="python -u bench.py --no-cpu-baseline --no-breakdown"
steps=("200:ob_base:$args")
for v in u2r128w6 u1r96w8 u2r128w5 u4w5 u2r128; do
  steps+=("200:ob_$v:SWH_LIB_PATH=swift_subtask_dev_amd/_exp/$v.so $args")
done
tools/gpu_steps.sh "${steps[@]}"
for f in base u2r128w6 u1r96w8 u2r128w5 u4w5 u2r128; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ob_$f.log') if l.startswith('{')][-1]); print('$f', d['value'], d['kernels']['density_ms'], d['kernels']['force_ms'], 'reuse', d['step_lists_reused']['density_ms'])" || true; done
