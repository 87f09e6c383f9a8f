#!/bin/bash
# Config-5 stand-in: overlap mode x gravity stream priority A/B.
export TMPDIR=/tmp
for m in async thread; do for p in 1 0; do
  SWH_COSMO_OVERLAP=$m SWH_GRAV_STREAM_PRIORITY=$p timeout -k 10 200 python bench.py --workload cosmo --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/cosmo_$m$p.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/cosmo_$m$p.log').read().strip().splitlines()[-1]); s=d['step_ms']; print('$m prio=$p', 'h %.3f g %.3f both %.3f gain %.3f' % (s['hydro_alone'], s['gravity_alone'], s['overlapped'], s['overlap_gain']), '%.4g' % d['value'])"
done; done
