#!/bin/bash
# round-2 closing set after the walk changes: GPU suite + smoke, bench + kernel
# trace + PMC traffic, SQ passes, TA busy of the walks
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "600:t_all:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" || exit $?
bash tools/profile_round.sh r02d || exit $?
KREGEX="list_build|walk_kernel" bash tools/pmc_passes.sh gpurun_out/r02d_pmc_sq || exit $?
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr GRBM_GUI_ACTIVE --kernel-include-regex "list_build|walk_kernel" \
  -d gpurun_out/r02d_ta -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-breakdown \
  > gpurun_out/r02d_ta.log 2>&1
echo "ta rc=$?"
