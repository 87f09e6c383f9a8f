#!/bin/bash
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread"
