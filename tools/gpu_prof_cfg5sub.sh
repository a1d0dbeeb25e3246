#!/usr/bin/env bash
# GPU box: kernel-trace summary of cfg5's chr21 (per-position) with exact
# block reuse off (STARCH_DEDUPE=0): where the doubling rounds spend their time.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/prof5
cd /tmp && export TMPDIR=/tmp
export STARCH_DEDUPE=0
timeout -k 10 300 python3 $ROOT/bench.py --kind 2 --chroms ${CHROMS:-13} --steps 1 --warmup 1 --no-cpu-baseline --no-e2e \
    > $ROOT/gpurun_out/prof5/bench.json 2> $ROOT/gpurun_out/prof5/bench.err || { tail -20 $ROOT/gpurun_out/prof5/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof5/tr -o run --output-format csv -- \
    python3 $ROOT/bench.py --kind 2 --chroms ${CHROMS:-13} --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-verify \
    > $ROOT/gpurun_out/prof5/prof.log 2>&1 || { tail -20 $ROOT/gpurun_out/prof5/prof.log; exit 1; }
python3 -c "import json;d=json.load(open('$ROOT/gpurun_out/prof5/bench.json'));print(d['ms_per_step'],d['stage_ms'],d['bwt'],d['verify'])"
find $ROOT/gpurun_out/prof5 -name '*kernel_stats*'
