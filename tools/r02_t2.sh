#!/bin/bash
tools/gpu_steps.sh \
 "600:t_sorted:python -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k 'sorted_oracle'" \
 "900:t_all:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300:grav:python -u bench.py --workload grav --n 256 --steps 3 --warmup 1"
