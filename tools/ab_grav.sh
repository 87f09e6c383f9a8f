#!/bin/bash
# gravity P2P A/B: parity of the batch P2P, then the config-4 bench
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:t_grav:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mpole.py tests/test_gpu_tree.py -x -q --timeout 120 --timeout-method thread -k 'grav or p2p or mpole or tree or P2P'" \
 "400:bgrav:python -u bench.py --workload grav --n 256 --steps 5 --warmup 1"
python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bgrav.log') if l.startswith('{')][-1]); print('bgrav', d['value'], d['ms_per_step'], d['roofline']['frac'])"
