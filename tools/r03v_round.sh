#!/bin/bash
# After striping the counted launches' atomics: GPU suite + smoke, then the
# headline profile (bench line, kernel trace, FETCH/WRITE PMC).
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" || exit $?
grep -q " passed" gpurun_out/t_all.log && ! grep -q " failed" gpurun_out/t_all.log || exit 1
KREGEX="list_build|walk_kernel|overflow_kernel|posf_kernel|list_prep|cell_reach|init_kernel|reset_acc" \
  tools/profile_round.sh r03v || exit $?
