#!/bin/bash
# Re-entry baseline: full GPU suite + smoke on HEAD, headline and cosmo lines.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "400:bench:python bench.py" \
 "300:bcosmo:python bench.py --workload cosmo --steps 10 --warmup 3"
