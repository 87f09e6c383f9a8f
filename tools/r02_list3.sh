#!/bin/bash
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --list-skin 0"
tools/gpu_steps.sh \
 "400:t_box:python -u -m pytest tests/test_dosub.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'box or clustered or periodic or dosub'" \
 "150:b7s0:$B" \
 "150:d1:$B --diag-mode 1" \
 "150:d2:$B --diag-mode 2"
bash tools/r02_trace.sh s0c --list-skin 0
python3 tools/bench_table.py b7s0 d1 d2
