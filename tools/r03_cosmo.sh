#!/bin/bash
# the config-5 stand-in (cosmo) with a kernel trace (csv stats)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:cosmo_trace:rocprofv3 --kernel-trace --stats -d gpurun_out/cosmo_trace -o run --output-format csv -- python -u bench.py --workload cosmo --steps 3 --warmup 1 --no-cpu-baseline"
