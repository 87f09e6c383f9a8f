#!/bin/bash
export TMPDIR=/tmp
tools/gpu_steps.sh "300:t_async:python -u -m pytest tests/test_gpu_async.py tests/test_gpu_threads.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider"
