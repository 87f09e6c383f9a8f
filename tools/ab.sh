#!/bin/bash
# A/B bench matrix: each arg "name:extra bench flags"; each run has its own
# time limit and the script stops at the first crash/timeout (tools/gpu_steps.sh).
specs=()
for a in "$@"; do n="${a%%:*}"; f="${a#*:}"; specs+=("150:$n:python bench.py --no-cpu-baseline --steps 10 $f"); done
exec tools/gpu_steps.sh "${specs[@]}"
