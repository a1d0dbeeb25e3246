#!/usr/bin/env bash
# GPU box: hardware-counter passes over a reduced bench run (one rocprofv3
# --pmc pass per counter set, each under its own time limit; --kernel-trace
# only, never combined with other trace domains).  Output: gpurun_out/pmc/<name>/
#   PASSES="sq1 sq2 fetch write" (default all), LINES=<bench --lines> (default 20M), KIND=<bench --kind>
set -o pipefail
mkdir -p gpurun_out/pmc
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
# one encoder lane (starch_set_lanes): per-kernel durations and counters not
# shared with a concurrent lane, and bench.py then runs no extra one-lane steps
# (the steps traced are exactly the ones asked for)
export STARCH_DEV_LANES=${STARCH_DEV_LANES:-1}
LINES=${LINES:-20000000}
PASSES=${PASSES:-sq1 sq2 fetch write}
run() {   # name, counters...
  local name=$1; shift
  timeout -s KILL ${TP:-120} rocprofv3 --kernel-trace --pmc "$@" -d $ROOT/gpurun_out/pmc/$name -o run \
      --output-format csv -- python3 $ROOT/bench.py --steps 1 --warmup 0 --kind ${KIND:-0} --lines $LINES --no-cpu-baseline --no-verify --no-e2e \
      > $ROOT/gpurun_out/pmc/$name.log 2>&1
}
rc=0
for p in $PASSES; do
  case $p in
    sq1) run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES ;;
    sq2) run sq2 SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS ;;
    fetch) run fetch FETCH_SIZE ;;
    write) run write WRITE_SIZE ;;
  esac
  rc=$?
  [ $rc -eq 0 ] || break
done
ls $ROOT/gpurun_out/pmc
exit $rc
