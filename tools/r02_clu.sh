#!/bin/bash
tools/gpu_steps.sh \
 "600:t_clu:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k 'clustered'"
