#!/bin/bash
tools/gpu_steps.sh \
 "600:t_27:python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k 'adapter_vs_f64'"
