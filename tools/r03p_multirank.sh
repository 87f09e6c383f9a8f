#!/bin/bash
# Multi-rank rehearsal on the one GPU over gloo (the driver's N>1 runs use
# RCCL, one GPU per rank): the headline split at 2 and 4 ranks, the config-5
# split at 2 ranks (bench.py spawns the ranks itself for --gpus N).
export TMPDIR=/tmp SWH_BENCH_BACKEND=gloo
tools/gpu_steps.sh \
 "300:mr2:python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline" \
 "300:mr4:python bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline" \
 "300:cosmo2:python bench.py --gpus 2 --workload cosmo --steps 5 --warmup 2 --no-cpu-baseline"
for f in mr2 mr4 cosmo2; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print('$f', d['n_gpus'], '%.4g' % d['value'], d['ms_per_step'], d['config'].get('density_interactions_per_step'), d['config'].get('hydro_interactions_per_step'))"; done
