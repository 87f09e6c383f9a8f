#!/bin/bash
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
tools/gpu_steps.sh \
 "400:t_box:python -u -m pytest tests/test_dosub.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'box or clustered or periodic or dosub'" \
 "150:b7s0:$B --list-skin 0" \
 "150:b7:$B"
bash tools/r02_trace.sh s0b --list-skin 0
python3 tools/bench_table.py b7s0 b7
