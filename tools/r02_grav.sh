#!/bin/bash
tools/gpu_steps.sh \
 "400:t_grav:python -u -m pytest tests/test_gpu_parity.py tests/test_dosub.py -x -q --timeout 300 --timeout-method thread -k 'grav or potential or dosub'" \
 "300:grav:python bench.py --workload grav --n 256 --steps 3 --warmup 1"
tail -1 gpurun_out/grav.log
