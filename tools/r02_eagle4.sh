#!/bin/bash
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300:e0:python -u bench.py --workload eagle --steps 10 --warmup 2" \
 "300:sedov:python -u bench.py --no-cpu-baseline"
