#!/bin/bash
export TMPDIR=/tmp
tools/gpu_steps.sh "300:t_gt:python -u -m pytest tests/test_gpu_grav_tasks.py tests/test_gpu_tree.py tests/test_gpu_mpole.py tests/test_grav_decomp.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider"
