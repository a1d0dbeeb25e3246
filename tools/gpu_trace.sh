#!/usr/bin/env bash
# GPU box: full kernel + memory-copy trace (every dispatch and copy, not just
# the summary) of one bench step: gpurun_out/trace/run_kernel_trace.csv and
# run_memory_copy_trace.csv.  BENCH_ARGS overrides the bench arguments.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/trace
cd /tmp && export TMPDIR=/tmp
BA=${BENCH_ARGS:---steps 1 --warmup 1}
timeout -k 10 ${TP:-300} rocprofv3 --kernel-trace --memory-copy-trace -d $ROOT/gpurun_out/trace -o run \
    --output-format csv -- python3 $ROOT/bench.py $BA --no-cpu-baseline --no-verify --no-e2e \
    > $ROOT/gpurun_out/trace.log 2>&1 || { tail -20 $ROOT/gpurun_out/trace.log; exit 1; }
find $ROOT/gpurun_out/trace -name '*.csv'
