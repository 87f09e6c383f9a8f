#!/bin/bash
# Full GPU suite (new physics / threading / drift tests first), then smoke.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "600:t_new:python -u -m pytest tests/test_gpu_physics.py tests/test_gpu_threads.py tests/test_gpu_drift.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread" \
 "900:t_all:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
