#!/bin/bash
# gravity parity, the cosmo stand-in, then its kernel trace
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:t_tree:python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_mpole.py tests/test_mesh.py tests/test_gpu_parity.py -k grav -x -q --timeout 120 --timeout-method thread" \
 "300:cosmo:python -u bench.py --workload cosmo --steps 5 --warmup 2 --no-cpu-baseline" \
 "300:cosmo_trace:rocprofv3 --kernel-trace --stats -d gpurun_out/cosmo_trace -o run --output-format csv -- python -u bench.py --workload cosmo --steps 3 --warmup 1 --no-cpu-baseline"
