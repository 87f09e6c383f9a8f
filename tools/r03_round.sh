#!/bin/bash
# GPU suite + smoke, then the default bench line and the grav line.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "400:bench:python bench.py" \
 "400:bgrav:python bench.py --workload grav --n 256 --steps 3 --warmup 1" || exit $?
tail -c 2500 gpurun_out/bench.log; echo; tail -c 1500 gpurun_out/bgrav.log
