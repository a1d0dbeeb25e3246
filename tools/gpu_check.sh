#!/usr/bin/env bash
# GPU box: selected test files (FILES), then the whole -m gpu suite, then one
# bench line.  Each GPU step has its own time limit; a failure ends the run.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PT="python -u -m pytest -x --timeout ${TT:-200} --timeout-method thread"
if [ -n "${FILES:-}" ]; then
  timeout -k 10 ${T0:-600} $PT -v $FILES > gpurun_out/t_new.log 2>&1 || { tail -30 gpurun_out/t_new.log; exit 1; }
  tail -3 gpurun_out/t_new.log
fi
if [ -z "${NOALL:-}" ]; then
  timeout -k 10 ${T1:-900} $PT -q -m gpu tests > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
  tail -3 gpurun_out/t_all.log
fi
if [ -z "${NOBENCH:-}" ]; then
  timeout -k 10 ${TB:-600} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
