#!/bin/bash
# Gravity parity suites, then the 256^3 P2P line and the cosmo line.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400:t_grav:python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_mpole.py tests/test_grav_decomp.py tests/test_gpu_parity.py -k 'grav or Potential or tree or mpole or m2p or owned' -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "300:bgrav:python bench.py --workload grav --n 256 --steps 3 --warmup 1 --no-cpu-baseline" \
 "300:bcosmo:python bench.py --workload cosmo --steps 10 --warmup 3 --no-cpu-baseline" || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bgrav.log').read().strip().splitlines()[-1]); print('grav', '%.4g' % d['value'], d['ms_per_step'], d['roofline']['frac'])"
python -c "import json; d=json.loads(open('gpurun_out/bcosmo.log').read().strip().splitlines()[-1]); print('cosmo', '%.4g' % d['value'], d['step_ms'], d['gravity_phase_ms_rank0'])"
