#!/bin/bash
tools/gpu_steps.sh \
 "600:eagle:python -u bench.py --workload eagle --steps 5 --warmup 1"
