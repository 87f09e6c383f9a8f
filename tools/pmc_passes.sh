#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, kernel-trace
# only; no runtime/sys trace domains are combined with --pmc).
# usage: KREGEX=<kernel regex> BENCH_ARGS="..." tools/pmc_passes.sh <outdir>
out="$1"; shift
mkdir -p "$out"
export TMPDIR=/tmp
KREGEX="${KREGEX:-list_build|walk_kernel|tile|loop_kernel|p2p_kernel}"
run() {
  local name="$1"; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KREGEX" \
    -d "$out/$name" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS \
    > "$out/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit $?
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH || exit $?
run tcc1 FETCH_SIZE || exit $?
run tcc2 WRITE_SIZE || exit $?
run tcc3 TCC_HIT_sum TCC_MISS_sum || exit $?
python3 tools/pmc_summary.py "$out"
