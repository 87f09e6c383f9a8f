#!/bin/bash
# asynchronous drift: drift tests, the whole GPU suite, then the bench with its step breakdown
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:t_drift:python -u -m pytest tests/test_gpu_drift.py -x -q --timeout 120 --timeout-method thread" \
 "600:t_all:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "300:bench:python -u bench.py --no-cpu-baseline"
python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench.log') if l.startswith('{')][-1]); print(d['value'], json.dumps(d['step_breakdown']))"
