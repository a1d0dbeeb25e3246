#!/usr/bin/env bash
# GPU box (round 6 dev): cfg5 with and without block reuse, + kernel stats of the no-reuse step
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
ROOT=$PWD
timeout -k 10 600 python bench.py --kind 2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/cfg5.json 2> $O/cfg5.err || { tail -20 $O/cfg5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg5.json'));print('cfg5', d['ms_per_step'], d['value'], d['verify']['match'], d['stage_ms'])"
STARCH_DEDUPE=0 timeout -k 10 900 python bench.py --kind 2 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $O/cfg5_nd.json 2> $O/cfg5_nd.err || { tail -20 $O/cfg5_nd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg5_nd.json'));print('cfg5 nodedupe', d['ms_per_step'], d['value'], d['verify']['match'], d['stage_ms'])"
if [ "${PROF:-1}" = 1 ]; then
( cd /tmp && export TMPDIR=/tmp STARCH_DEDUPE=0 && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof_cfg5nd -o run --output-format csv -- \
    python3 $ROOT/bench.py --kind 2 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-verify > $ROOT/$O/prof_cfg5nd.log 2>&1 ) || { tail -5 $O/prof_cfg5nd.log; exit 1; }
f=$(find $O/prof_cfg5nd -name '*kernel_stats.csv' | head -1)
python3 tools/kstats.py "$f" 1 30
fi
