#!/bin/bash
# sharded tree gravity: GPU tests, the cosmo line at N=1 and a 2-rank gloo
# rehearsal on the one GPU (the driver's N>1 runs use RCCL, one GPU per rank)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:t_shard:python -u -m pytest tests/test_grav_decomp.py tests/test_gpu_tree.py -x -q -rf --timeout 200 --timeout-method thread" \
 "300:cosmo1:python -u bench.py --workload cosmo --steps 10 --warmup 3 --no-cpu-baseline" \
 "300:cosmo2:SWH_BENCH_BACKEND=gloo python -u bench.py --gpus 2 --workload cosmo --steps 10 --warmup 3"
grep -o '"value[^,]*\|"step_ms[^}]*' gpurun_out/cosmo1.log gpurun_out/cosmo2.log
