#!/bin/bash
tools/gpu_steps.sh \
 "600:t_all:python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300:bench:python bench.py" \
 "300:grav:python bench.py --workload grav --n 256 --steps 3 --warmup 1"
python3 tools/bench_table.py bench
tail -1 gpurun_out/grav.log
