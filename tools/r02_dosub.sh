#!/bin/bash
tools/gpu_steps.sh \
 "300:t_dosub:python -u -m pytest tests/test_dosub.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'dosub or 27cells or force_pair or potential or unsorted'"
BENCH_ARGS="--list-skin 0" bash tools/pmc_passes.sh gpurun_out/pmc_s0
