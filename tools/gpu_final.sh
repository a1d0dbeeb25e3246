#!/usr/bin/env bash
# GPU box, end of a round: every GPU test and the smoke check; the block-sort
# HBM traffic from two PMC passes (FETCH_SIZE, WRITE_SIZE) over one cfg2 step,
# stamped with these sources; then the bench line (which attaches that
# traffic) and the rocprofv3 kernel-trace summary of the same command.
# Outputs under gpurun_out/: gpu_tests.log, pmc/, pmc_k_bwt.json, bench.json,
# prof/run_kernel_stats.csv.  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
PASSES="fetch write" LINES=100000000 TP=150 bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 1; }
LINES=100000000 python tools/pmc_bwt_traffic.py gpurun_out/pmc gpurun_out/pmc_k_bwt.json || exit 1
cp gpurun_out/pmc_k_bwt.json profiles/pmc_k_bwt.json
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
BENCH_ARGS="--steps 2 --warmup 1" TP=300 bash tools/gpu_prof.sh > /dev/null || exit 1
