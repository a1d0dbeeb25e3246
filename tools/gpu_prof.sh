#!/usr/bin/env bash
# GPU box: rocprofv3 kernel-trace summary of bench.py (cfg2 unless BENCH_ARGS),
# then optional PMC passes (PASSES="sq1 sq2 fetch write"), each its own run
# under its own time limit.  Output: gpurun_out/prof/, gpurun_out/pmc/<pass>/
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/prof $ROOT/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
# one encoder lane (starch_set_lanes): per-kernel durations and counters not
# shared with a concurrent lane, and bench.py then runs no extra one-lane steps
# (the steps traced are exactly the ones asked for)
export STARCH_DEV_LANES=${STARCH_DEV_LANES:-1}
BA=${BENCH_ARGS:---steps 2 --warmup 1}
timeout -k 10 ${TP:-300} rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof -o run --output-format csv -- \
    python3 $ROOT/bench.py $BA --no-cpu-baseline --no-verify --no-e2e > $ROOT/gpurun_out/prof.log 2>&1 \
    || { tail -20 $ROOT/gpurun_out/prof.log; exit 1; }
for p in ${PASSES:-}; do
  case $p in
    sq1) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" ;;
    sq2) C="SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS" ;;
    fetch) C="FETCH_SIZE" ;;
    write) C="WRITE_SIZE" ;;
    *) continue ;;
  esac
  timeout -s KILL ${TPMC:-150} rocprofv3 --kernel-trace --pmc $C -d $ROOT/gpurun_out/pmc/$p -o run --output-format csv -- \
      python3 $ROOT/bench.py --steps 1 --warmup 0 ${PMC_ARGS:-} --no-cpu-baseline --no-verify --no-e2e \
      > $ROOT/gpurun_out/pmc/$p.log 2>&1 || { echo "pmc pass $p failed"; tail -5 $ROOT/gpurun_out/pmc/$p.log; exit 1; }
done
find $ROOT/gpurun_out/prof -name '*kernel_stats*'
