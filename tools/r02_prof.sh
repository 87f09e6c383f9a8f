#!/bin/bash
# round-2 profile set: bench + kernel trace + FETCH/WRITE passes + SQ passes
export TMPDIR=/tmp
bash tools/profile_round.sh r02a || exit $?
KREGEX="list_build|walk_kernel" bash tools/pmc_passes.sh gpurun_out/r02a_pmc_sq
