#!/usr/bin/env bash
# GPU box: FETCH_SIZE / WRITE_SIZE calibration (tools/probes/fetch_calib.hip,
# prebuilt as dbgbuild/fetch_calib) -> gpurun_out/fetch_calib.json
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/fcal
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for p in fetch write; do
  C=FETCH_SIZE; [ $p = write ] && C=WRITE_SIZE
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $O/$p -o run --output-format csv -- $ROOT/dbgbuild/fetch_calib \
      > $O/$p.log 2>&1 || { echo "pass $p failed"; tail -5 $O/$p.log; exit 1; }
done
python3 $ROOT/tools/fetch_calib_summary.py $O $ROOT/gpurun_out/fetch_calib.json
