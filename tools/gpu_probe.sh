#!/usr/bin/env bash
# GPU box: one probe of bench.py (BENCH_ARGS) -- its JSON line, stderr and,
# unless NOPROF=1, the rocprofv3 kernel-trace summary of the same command.
# ENVS: extra environment for the bench process (e.g. STARCH_BWT_DEBUG=1).
# Output: gpurun_out/probe/<TAG>.{json,err,csv}
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-probe}
O=$ROOT/gpurun_out/probe
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
BA=${BENCH_ARGS:---steps 2 --warmup 1}
env $ENVS timeout -k 10 ${TB:-300} python3 $ROOT/bench.py $BA --no-cpu-baseline --no-e2e > $O/$TAG.json 2> $O/$TAG.err \
    || { tail -20 $O/$TAG.err; exit 1; }
cat $O/$TAG.json
if [ -z "${NOPROF:-}" ]; then
  [ -n "$ENVS" ] && export $ENVS
  rm -rf $O/prof_$TAG
  timeout -k 10 ${TP:-300} rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- \
      python3 $ROOT/bench.py $BA --no-cpu-baseline --no-verify --no-e2e > $O/$TAG.prof.log 2>&1 \
      || { tail -20 $O/$TAG.prof.log; exit 1; }
  f=$(find $O/prof_$TAG -name '*kernel_stats.csv' | head -1)
  cp "$f" $O/$TAG.kstats.csv
  rm -rf $O/prof_$TAG
  python3 $ROOT/tools/kstats.py $O/$TAG.kstats.csv ${KSTEPS:-3} 25
fi
