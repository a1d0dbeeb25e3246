#!/usr/bin/env bash
# GPU box: hardware-counter passes over a reduced bench run (one rocprofv3
# --pmc pass per counter set, each under its own time limit; --kernel-trace
# only, never combined with other trace domains).  Output: gpurun_out/pmc/<name>/
set -o pipefail
mkdir -p gpurun_out/pmc
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
LINES=${LINES:-20000000}
run() {   # name, counters...
  local name=$1; shift
  timeout -s KILL ${TP:-120} rocprofv3 --kernel-trace --pmc "$@" -d $ROOT/gpurun_out/pmc/$name -o run \
      --output-format csv -- python3 $ROOT/bench.py --steps 1 --warmup 0 --lines $LINES --no-cpu-baseline \
      > $ROOT/gpurun_out/pmc/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES &&
run sq2 SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE
rc=$?
ls $ROOT/gpurun_out/pmc
exit $rc
