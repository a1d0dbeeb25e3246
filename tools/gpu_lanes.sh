#!/usr/bin/env bash
# GPU box: device-path encoder lanes (STARCH_DEV_LANES) A/B on cfg2, 1/8 of
# cfg2 and (CFG5=1) cfg5; bench lines -> gpurun_out/ln/<name>.json
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/ln
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {   # name env... -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e "$@" > $O/$name.json 2> $O/$name.err \
    || { tail -20 $O/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['ms_per_step'], d['value'], d['verify']['match'] if d.get('verify') else '-', d['stage_ms'])"
}
for L in ${LANES:-1 2}; do
  run cfg2_l$L STARCH_DEV_LANES=$L --
  run eighth_l$L STARCH_DEV_LANES=$L -- --lines 12500000 --steps 10 --warmup 3
done
if [ "${CFG5:-0}" = 1 ]; then
  for L in ${LANES:-1 2}; do run cfg5_l$L STARCH_DEV_LANES=$L -- --kind 2 --steps 2 --warmup 1; done
fi
