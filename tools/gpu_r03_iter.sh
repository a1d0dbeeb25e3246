#!/usr/bin/env bash
# GPU box, one development iteration: selected test files (FILES) first, then
# the whole -m gpu suite, then the bench line and a kernel-trace summary of the
# same command (gpurun_out/prof).  Each step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PT="python -u -m pytest -x --timeout ${TT:-300} --timeout-method thread"
if [ -n "${FILES:-}" ]; then
  timeout -k 10 ${T0:-900} $PT -v $FILES > gpurun_out/t_new.log 2>&1 || { tail -40 gpurun_out/t_new.log; exit 1; }
  tail -3 gpurun_out/t_new.log
fi
if [ -z "${NOALL:-}" ]; then
  timeout -k 10 ${T1:-900} $PT -q -m gpu tests > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
  tail -2 gpurun_out/t_all.log
fi
timeout -k 10 ${TB:-400} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
BENCH_ARGS="--steps 2 --warmup 1" TP=300 bash tools/gpu_prof.sh > /dev/null || exit 1
python3 tools/kstats.py gpurun_out/prof/run_kernel_stats.csv 3 30
