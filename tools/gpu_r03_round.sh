#!/usr/bin/env bash
# GPU box, one round-3 iteration: every GPU test, the cfg2 bench line, the
# kernel trace of the same command (gpurun_out/prof), the transform alone
# (cfg2, cfg4), the cfg4 bench line, then optional sweep VARIANTS and an
# e2e host timeline (E2E=1).  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PT="python -u -m pytest -x --timeout ${TT:-300} --timeout-method thread"
if [ -z "${NOTESTS:-}" ]; then
  timeout -k 10 ${T1:-1000} $PT -q -m gpu tests > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
  tail -2 gpurun_out/t_all.log
fi
timeout -k 10 ${TB:-400} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
BENCH_ARGS="--steps 2 --warmup 1" TP=300 bash tools/gpu_prof.sh > /dev/null || exit 1
python3 tools/kstats.py gpurun_out/prof/run_kernel_stats.csv 3 30
python3 tools/gaps.py gpurun_out/prof/run_kernel_trace.csv 40 | tail -25
for k in 0 1; do timeout -k 10 120 python tools/tf_bench.py --kind $k --lines $([ $k = 0 ] && echo 100000000 || echo 50000000) 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1; done
timeout -k 10 400 python bench.py --kind 1 --lines 50000000 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { tail -30 gpurun_out/bench_cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_cfg4.json')); print('cfg4', d['value'], d['ms_per_step'], d['stage_ms'], d['verify'])"
if [ -n "${VARIANTS:-}" ]; then bash tools/gpu_sweep.sh || exit 1; fi
if [ -n "${E2E:-}" ]; then NOTEST=1 VARIANTS="2:8" bash tools/gpu_r03_e2e.sh || exit 1; fi
