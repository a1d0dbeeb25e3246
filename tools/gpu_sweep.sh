#!/usr/bin/env bash
# GPU box: bench.py stage times for each library variant in VARIANTS
# (starch_amd/_sweep/<v>/libstarch_amd.so; "base" = starch_amd/_build).
set -o pipefail
mkdir -p gpurun_out/sweep
for v in ${VARIANTS:-base}; do
  lib=starch_amd/_sweep/$v/libstarch_amd.so
  [ "$v" = base ] && lib=starch_amd/_build/libstarch_amd.so
  STARCH_AMD_LIB=$lib timeout -k 10 ${TB:-200} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} --no-cpu-baseline --no-verify --no-e2e \
     > gpurun_out/sweep/$v.json 2> gpurun_out/sweep/$v.err || { echo "variant $v failed"; tail -5 gpurun_out/sweep/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep/$v.json')); print('$v', d['ms_per_step'], d['stage_ms'])"
done
