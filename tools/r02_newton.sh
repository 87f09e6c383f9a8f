#!/bin/bash
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "200:b1:python -u bench.py --no-cpu-baseline" \
 "300:grav:python -u bench.py --workload grav --n 256 --steps 3 --warmup 1"
