#!/usr/bin/env bash
# GPU box: one rocprofv3 --pmc pass of L2 (TCC) hit/miss and memory-side read
# request counters over one bench step (dev tool).  Output: gpurun_out/pmc/tcc/
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL ${TP:-150} rocprofv3 --kernel-trace --pmc ${CTRS:-TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum} \
    -d $ROOT/gpurun_out/pmc/${NAME:-tcc} -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 1 --warmup 0 ${PMC_ARGS:-} --no-cpu-baseline --no-verify --no-e2e \
    > $ROOT/gpurun_out/pmc/${NAME:-tcc}.log 2>&1 || { tail -5 $ROOT/gpurun_out/pmc/${NAME:-tcc}.log; exit 1; }
