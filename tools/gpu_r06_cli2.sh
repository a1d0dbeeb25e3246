#!/usr/bin/env bash
# GPU box (round 6 dev): pipe batch sizes, teardown cost, a cold CLI timeline
set -o pipefail
O=gpurun_out/cli6
mkdir -p $O
F=${TMPDIR:-/tmp}/cfg2_cli6.bed
trap 'rm -f $F $O/*.starch' EXIT
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.')
import starch_amd
open('$F','wb').write(starch_amd.gen_bed(0, 100000000))" || exit 1
ms() { echo $(( ($2 - $1) / 1000000 )); }
stat1() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print({k:d[k] for k in ('create_s','setup_s','end_s','wall_s','after_setup_mb_s') if k in d})"; }
for b in 256 128 64 128 64 32; do
  a=$(date +%s%N); cat $F | timeout -k 10 60 starch_amd/_build/starch3 --stats --batch-mb $b > $O/pipe.starch 2> $O/pipe.err || { tail -5 $O/pipe.err; exit 1; }; c=$(date +%s%N)
  echo "pipe batch=$b wall $(ms $a $c) ms $(stat1 $O/pipe.err)"
done
for t in 0 1; do
  a=$(date +%s%N); STARCH_CLI_TEARDOWN=$t timeout -k 10 60 starch_amd/_build/starch3 --stats < $F > $O/file.starch 2> $O/file.err || { tail -5 $O/file.err; exit 1; }; c=$(date +%s%N)
  echo "file teardown=$t wall $(ms $a $c) ms $(grep teardown $O/file.err) $(stat1 $O/file.err)"
  a=$(date +%s%N); cat $F | STARCH_CLI_TEARDOWN=$t timeout -k 10 60 starch_amd/_build/starch3 --stats --batch-mb 64 > $O/pipe.starch 2> $O/pipe.err || { tail -5 $O/pipe.err; exit 1; }; c=$(date +%s%N)
  echo "pipe64 teardown=$t wall $(ms $a $c) ms $(grep teardown $O/pipe.err) $(stat1 $O/pipe.err)"
done
cmp $O/file.starch $O/pipe.starch || exit 1
R=$PWD
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $R/$O/ktr -o run --output-format csv -- $R/starch_amd/_build/starch3 --stats < $F > $R/$O/file.starch 2> $R/$O/ktr.err ) || { tail -5 $O/ktr.err; exit 1; }
find $O/ktr -name '*kernel_trace.csv' | head -1
