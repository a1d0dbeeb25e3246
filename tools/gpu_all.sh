#!/usr/bin/env bash
# GPU box: parity tests, then (only if they pass) the bench line and an
# optional rocprofv3 kernel-trace summary.  Every GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${T1:-900} python -m pytest tests -m gpu ${XFLAG--x} -q ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${TB:-900} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
tail -4 gpurun_out/bench.err
if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 ${TP:-900} rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-e2e > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
fi
