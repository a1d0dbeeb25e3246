#!/usr/bin/env bash
# GPU box: the CLI's set-up split (--stats: create_s = device contexts open,
# setup_s = until the first input byte is read) on the cfg2 input as a file,
# three runs each of `starch3 < file` and of the hpp example.
set -o pipefail
O=gpurun_out/cli
mkdir -p $O
trap 'rm -f $O/a.starch $O/b.starch ${TMPDIR:-/tmp}/cfg2_cli.bed' EXIT
F=${TMPDIR:-/tmp}/cfg2_cli.bed
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.')
import starch_amd
open('$F','wb').write(starch_amd.gen_bed(0, 100000000))" || exit 1
for v in "1 eager 256" "1 eager 256" "1 eager 256"; do
  set -- $v
  a=$(date +%s%N)
  STARCH_CLI_MAP=$1 STARCH_PIN=$2 timeout -k 10 60 starch_amd/_build/starch3 --stats --batch-mb $3 < $F > $O/a.starch 2> $O/cli.err || { cat $O/cli.err; exit 1; }
  b=$(date +%s%N)
  echo "map=$1 pin=$2 batch=$3 external wall $(( (b - a) / 1000000 )) ms $(python3 -c "import json;d=json.loads(open('$O/cli.err').read().strip().splitlines()[-1]);print({k:d[k] for k in ('premain_s','create_s','begin_s','encode_s','end_s','wall_s','after_setup_mb_s')})")"
done
for i in 1 2; do
  a=$(date +%s%N)
  timeout -k 10 60 starch_amd/_build/starch3_hpp_example --hook < $F > $O/b.starch 2> $O/hook_$i.err || { cat $O/hook_$i.err; exit 1; }
  b=$(date +%s%N)
  echo "hook external wall $(( (b - a) / 1000000 )) ms"
done
cmp $O/a.starch $O/b.starch && echo identical
STARCH_TRACE=1 starch_amd/_build/starch3 --stats < $F > $O/a.starch 2> $O/trace.err; tail -40 $O/trace.err
rm -f $F $O/a.starch $O/b.starch
