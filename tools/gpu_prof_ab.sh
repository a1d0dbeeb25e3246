#!/usr/bin/env bash
# GPU box: kernel-trace summaries of bench.py under two environments (A/B):
# gpurun_out/ab/a and gpurun_out/ab/b.  ENV_A / ENV_B: "VAR=value ..." lists.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
BA=${BENCH_ARGS:---steps 2 --warmup 1}
for side in a b; do
  mkdir -p $ROOT/gpurun_out/ab/$side
  E=ENV_${side^^}
  ( export ${!E}; timeout -k 10 ${TP:-300} rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/ab/$side -o run \
      --output-format csv -- python3 $ROOT/bench.py $BA --no-cpu-baseline --no-verify --no-e2e \
      > $ROOT/gpurun_out/ab/$side.log 2>&1 ) || { tail -20 $ROOT/gpurun_out/ab/$side.log; exit 1; }
done
find $ROOT/gpurun_out/ab -name '*kernel_stats*'
