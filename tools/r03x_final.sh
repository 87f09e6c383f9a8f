#!/bin/bash
# Final check of the round's tree: GPU suite, smoke, default bench line.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300:r03x_bench:python bench.py" || exit $?
