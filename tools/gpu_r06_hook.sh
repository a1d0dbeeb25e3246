#!/usr/bin/env bash
# GPU box (round 6 dev): where the hpp hook's time goes (STARCH_HOOK_TRACE=1), cfg2 as a file
set -o pipefail
O=gpurun_out/cli6
mkdir -p $O
F=${TMPDIR:-/tmp}/cfg2_hook.bed
trap 'rm -f $F $O/*.starch' EXIT
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.')
import starch_amd
open('$F','wb').write(starch_amd.gen_bed(0, 100000000))" || exit 1
ms() { echo $(( ($2 - $1) / 1000000 )); }
for i in 1 2 3; do
  a=$(date +%s%N); STARCH_HOOK_TRACE=1 STARCH_BZ_TRACE=1 timeout -k 10 60 starch_amd/_build/starch3_hpp_example --hook < $F > $O/h.starch 2> $O/h.err || { tail -5 $O/h.err; exit 1; }; b=$(date +%s%N)
  echo "hook wall $(ms $a $b) ms"; grep -E "trace|bz" $O/h.err | tail -3
done
for i in 1 2; do
  a=$(date +%s%N); timeout -k 10 60 starch_amd/_build/starch3_hpp_example < $F > $O/p.starch 2> $O/p.err || { tail -5 $O/p.err; exit 1; }; b=$(date +%s%N)
  echo "hpp wall $(ms $a $b) ms"
done
cmp $O/h.starch $O/p.starch && echo identical
