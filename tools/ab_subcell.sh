export TMPDIR=/tmp
for sb in 0 3 0 3; do
  SWH_SUBCELL_BITS=$sb timeout -k 10 200 python bench.py --no-cpu-baseline --no-breakdown --steps 20 > gpurun_out/ab1_$sb.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab1_$sb.log').read().strip().splitlines()[-1]); print('sb=$sb', d['ms_per_step'], d['kernels']['density_ms'], d['kernels']['force_ms'], d['step_lists_reused']['density_ms'])"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "headline or box_chain or clustered" > gpurun_out/ab1_tests.log 2>&1; echo tests rc=$?; tail -3 gpurun_out/ab1_tests.log
