#!/bin/bash
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "600:eagle:python -u bench.py --workload eagle --steps 5 --warmup 1" \
 "400:sedov:python -u bench.py --no-cpu-baseline"
