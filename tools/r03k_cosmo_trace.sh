#!/bin/bash
# Kernel trace of the config-5 stand-in (hydro || gravity): busy time per stream.
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cosmo_trace -o run --output-format csv -- python bench.py --workload cosmo --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cosmo_trace.log 2>&1 || exit $?
tail -1 gpurun_out/cosmo_trace.log | cut -c1-300
