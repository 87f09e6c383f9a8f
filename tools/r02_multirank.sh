#!/bin/bash
# Rehearse bench.py's multi-rank path (strong split, halo refresh, max over
# ranks) with 2 and 4 ranks sharing the box's GPU over gloo (the driver's
# 8-GPU runs use RCCL, one GPU per rank).
export TMPDIR=/tmp SWH_BENCH_BACKEND=gloo
tools/gpu_steps.sh \
 "300:mr2:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1" \
 "300:mr4:python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 1"
for f in mr2 mr4; do python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print('$f', d['n_gpus'], d['value'], d['ms_per_step'], d['config'].get('density_interactions_per_step'), d['config'].get('decomposition'))"; done
