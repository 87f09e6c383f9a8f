#!/bin/bash
tools/gpu_steps.sh \
 "600:t_mp:python -u -m pytest tests/test_gpu_mpole.py -v --timeout 120 --timeout-method thread"
