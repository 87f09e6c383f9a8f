#!/bin/bash
# Run GPU steps in order; each step has its own time limit. A step that
# crashes (abort/segfault/timeout) ends the script: nothing else touches the
# GPU after a fault. Ordinary test failures (rc=1) do not stop later steps.
# usage: tools/gpu_steps.sh "<limit_s>:<name>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  limit="${spec%%:*}"; rest="${spec#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
  echo "== step $name (limit ${limit}s): $cmd"
  timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== step $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then
    echo "== stopping after crash/timeout in $name"; exit $rc
  fi
done
