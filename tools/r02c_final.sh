#!/bin/bash
# round-2 closing set: GPU suite + smoke, bench + kernel trace + PMC traffic, SQ passes
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "600:t_all:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" || exit $?
bash tools/profile_round.sh r02c || exit $?
KREGEX="list_build|walk_kernel" bash tools/pmc_passes.sh gpurun_out/r02c_pmc_sq
