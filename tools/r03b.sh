#!/bin/bash
# full GPU suite + smoke, the headline line, the grav 256^3 line with its
# kernel trace and FETCH/WRITE passes, the cosmo line with its CPU baseline
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900:t_all:python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200:smoke:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "400:bench:python bench.py" \
 "400:bgrav:python bench.py --workload grav --n 256 --steps 3 --warmup 1" \
 "300:grav_trace:rocprofv3 --kernel-trace --stats -d gpurun_out/grav_trace -o run --output-format csv -- python -u bench.py --workload grav --n 256 --steps 3 --warmup 1 --no-cpu-baseline" \
 "300:bcosmo:python bench.py --workload cosmo --steps 10 --warmup 3" || exit $?
KREGEX="p2p_kernel" BENCH_ARGS="--workload grav --n 256" bash -c '
out=gpurun_out/pmc_grav; mkdir -p $out
for pass in "tcc1 FETCH_SIZE" "tcc2 WRITE_SIZE"; do set -- $pass; name=$1; shift
timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KREGEX" -d $out/$name -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $out/$name.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py $out > gpurun_out/pmc_grav.txt'
