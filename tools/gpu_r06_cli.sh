#!/usr/bin/env bash
# GPU box (round 6 dev): whole-process costs of the CLI on cfg2.
#   exit_probe: HIP init + pinned + device memory, then _exit, timed outside
#   starch3 < file, cat file | starch3 (pipe reader on / off), each 3x, --stats
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
if [ "${EXIT:-1}" = 1 ]; then
for v in "0 0" "0 4096" "0 16384" "2048 0" "0 0 1" "0 16384 1"; do
  set -- $v
  a=$(date +%s%N); timeout -k 10 60 starch_amd/_build/exit_probe $1 $2 ${3:-0} 2> $O/ep.err || { cat $O/ep.err; exit 1; }; b=$(date +%s%N)
  echo "exit_probe pin_mb=$1 dev_mb=$2 teardown=${3:-0}: wall $(ms $a $b) ms | $(cat $O/ep.err | tr '\n' ' ')"
done
fi
stat1() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print({k:d[k] for k in d if k.endswith('_s') or k.endswith('mb_s')})"; }
for i in 1 2 3; do
  a=$(date +%s%N); timeout -k 10 60 starch_amd/_build/starch3 --stats < $F > $O/file.starch 2> $O/file.err || { tail -5 $O/file.err; exit 1; }; b=$(date +%s%N)
  echo "file  wall $(ms $a $b) ms $(stat1 $O/file.err)"
done
for pr in 1 1 1 0; do
  a=$(date +%s%N); cat $F | STARCH_CLI_PIPE=$pr timeout -k 10 60 starch_amd/_build/starch3 --stats > $O/pipe.starch 2> $O/pipe.err || { tail -5 $O/pipe.err; exit 1; }; b=$(date +%s%N)
  echo "pipe reader=$pr wall $(ms $a $b) ms $(stat1 $O/pipe.err)"
  cmp $O/file.starch $O/pipe.starch || { echo "pipe archive differs"; exit 1; }
done
a=$(date +%s%N); cat $F > /dev/null; b=$(date +%s%N); echo "cat > /dev/null $(ms $a $b) ms"
a=$(date +%s%N); cat $F | cat > /dev/null; b=$(date +%s%N); echo "cat | cat > /dev/null $(ms $a $b) ms"
echo identical
