#!/usr/bin/env bash
# GPU box (round 6 dev): the CLI's cold encode on cfg2 -- library trace and kernel timeline
set -o pipefail
O=$PWD/gpurun_out/cold
mkdir -p $O
F=/tmp/cfg2_cold.bed
trap 'rm -f $F $O/*.starch' EXIT
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.')
import starch_amd
open('$F','wb').write(starch_amd.gen_bed(0, 100000000))" || exit 1
STARCH_TRACE=1 timeout -k 10 60 starch_amd/_build/starch3 --stats < $F > $O/a.starch 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
tail -60 $O/trace.err | cut -c1-200
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/ktr -o run --output-format csv -- $R/starch_amd/_build/starch3 --stats < $F > $O/b.starch 2> $O/ktr.err || { tail -5 $O/ktr.err; exit 1; }
find $O/ktr -name '*.csv' | head
