#!/bin/bash
# A/B timing of bench.py variants on one GPU box (replaces the one-off
# tools/ab_*.sh and tools/r0[23]*.sh scripts of rounds 2-3; see git history).
# usage: tools/gpu_ab.sh <tag> "<bench args A>" "<bench args B>" [reps]
#   env: SWH_AB_ENV_A / SWH_AB_ENV_B = extra environment (e.g. SWH_LIB_PATH=...)
# Alternates A, B, A, B, ... (reps each); one line per run in
# gpurun_out/<tag>_summary.txt: variant, ms/step, density ms, force ms, value.
tag="$1"; A="$2"; B="$3"; reps="${4:-2}"
set -o pipefail
out=gpurun_out
mkdir -p $out
for r in $(seq 1 "$reps"); do
  for v in A B; do
    args=$A; envs=$SWH_AB_ENV_A
    if [ $v = B ]; then args=$B; envs=$SWH_AB_ENV_B; fi
    log="$out/${tag}_${v}${r}.log"
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-steady --no-breakdown --no-configs \
      $args > "$log" 2>&1 || exit $?
    tail -1 "$log" | python -c "
import json, sys
d = json.loads(sys.stdin.read()); k = d.get('kernels') or {}
print('$v', d['ms_per_step'], k.get('density_ms'), k.get('force_ms'), d['value'])" \
      >> "$out/${tag}_summary.txt" || exit $?
  done
done
cat "$out/${tag}_summary.txt"
