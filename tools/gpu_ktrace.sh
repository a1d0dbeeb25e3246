#!/usr/bin/env bash
# GPU box: kernel-trace summaries of bench.py for library variants (dev tool):
# VARIANTS="base v1 ..." (starch_amd/_sweep/<v>/libstarch_amd.so), one rocprofv3
# --kernel-trace --stats run each.  Output: gpurun_out/kt/<v>/
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  lib=$ROOT/starch_amd/_sweep/$v/libstarch_amd.so
  [ "$v" = base ] && lib=$ROOT/starch_amd/_build/libstarch_amd.so
  mkdir -p $ROOT/gpurun_out/kt/$v
  STARCH_AMD_LIB=$lib timeout -k 10 ${TP:-200} rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/kt/$v -o run \
      --output-format csv -- python3 $ROOT/bench.py ${BENCH_ARGS:---steps 2 --warmup 1} --no-cpu-baseline --no-verify --no-e2e \
      > $ROOT/gpurun_out/kt/$v.log 2>&1 || { echo "variant $v failed"; tail -5 $ROOT/gpurun_out/kt/$v.log; exit 1; }
done
