#!/usr/bin/env bash
# GPU box: per-encode fixed cost at cfg1 size (tools/small_cost.py), plain and
# under rocprofv3 --hip-trace --kernel-trace --stats (HIP calls per encode).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/small
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $ROOT/tools/small_cost.py ${REPS:-300} > $O/plain.json 2> $O/plain.err || { tail -20 $O/plain.err; exit 1; }
cat $O/plain.json
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 $ROOT/tools/small_cost.py 100 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name '*stats.csv'
