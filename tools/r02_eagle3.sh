#!/bin/bash
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300:e0:python -u bench.py --workload eagle --steps 5 --warmup 1" \
 "300:e15:python -u bench.py --workload eagle --steps 5 --warmup 1 --cell-scale 1.5" \
 "300:e2:python -u bench.py --workload eagle --steps 5 --warmup 1 --cell-scale 2" \
 "300:e3:python -u bench.py --workload eagle --steps 5 --warmup 1 --cell-scale 3" \
 "300:sedov:python -u bench.py --no-cpu-baseline"
