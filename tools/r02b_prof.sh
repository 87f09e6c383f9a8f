#!/bin/bash
# round-2 (second session) profile set: bench + kernel trace + FETCH/WRITE passes + SQ passes
export TMPDIR=/tmp
bash tools/profile_round.sh r02b || exit $?
KREGEX="list_build|walk_kernel" bash tools/pmc_passes.sh gpurun_out/r02b_pmc_sq
