#!/usr/bin/env bash
# GPU box: A/B kernel-trace summaries (base library vs a starch_amd/_sweep
# variant, VAR=<name>) on cfg2, then a small-input trace with the HIP runtime
# API (fixed per-encode costs: syncs, copies).  Each step has its own limit.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
ENV_A="STARCH_AMD_LIB=$ROOT/starch_amd/_build/libstarch_amd.so" \
ENV_B="STARCH_AMD_LIB=$ROOT/starch_amd/_sweep/${VAR:-nogather}/libstarch_amd.so" \
  TP=${TP:-200} bash $ROOT/tools/gpu_prof_ab.sh || exit 1
if [ -n "${SMALL:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  mkdir -p $ROOT/gpurun_out/small
  timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $ROOT/gpurun_out/small -o run \
      --output-format csv -- python3 $ROOT/bench.py --lines ${SMALL} --steps 20 --warmup 3 --no-cpu-baseline \
      --no-verify --no-e2e > $ROOT/gpurun_out/small.log 2>&1 || { tail -20 $ROOT/gpurun_out/small.log; exit 1; }
fi
