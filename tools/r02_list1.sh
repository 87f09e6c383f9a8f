#!/bin/bash
# round 2: first pair-list run: parity tests of the batch loops + bench A/B
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
tools/gpu_steps.sh \
 "300:t_box:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'box or clustered or periodic'" \
 "150:b7:$B" \
 "150:b7s0:$B --list-skin 0" \
 "150:b7s05:$B --list-skin 0.05" \
 "150:b7d1:$B --diag-mode 1" \
 "150:b5:$B --loop-variant 5"
python3 tools/bench_table.py b7 b7s0 b7s05 b7d1 b5
