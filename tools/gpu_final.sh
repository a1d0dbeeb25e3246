#!/usr/bin/env bash
# GPU box, end-of-round measurement package at the current sources, in two
# calls (each fits one gpurun limit):
#   PHASE=pmc    every GPU test and smoke(); stamped block-sort counters for
#                cfg2 and cfg4 (FETCH/WRITE_SIZE traffic, SQ wait/issue split)
#                plus SQ of every kernel for cfg2 -> gpurun_out/final/
#                (copy pmc_k_bwt*.json to profiles/ before PHASE=bench: the
#                bench line attaches them only when their stamp matches)
#   PHASE=bench  the cfg2 bench line (CPU baseline, e2e, streamed, CLI legs),
#                cfg4, cfg5 (CFG5=1), 1/8 of cfg2, cfg1 fixed cost, and the
#                rocprofv3 kernel-trace summaries of cfg2 and cfg4
# Each GPU step has its own time limit; a failure ends the run.
set -o pipefail
mkdir -p gpurun_out/final
export PYTHONUNBUFFERED=1
O=gpurun_out/final
if [ "${PHASE:-pmc}" = pmc ]; then
  if [ -z "${NOTESTS:-}" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
        || { tail -30 $O/gpu_tests.log; exit 1; }
    tail -2 $O/gpu_tests.log
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
    cat $O/smoke.log
  fi
  for w in cfg2 cfg4; do
    if [ $w = cfg2 ]; then K=0; L=100000000; S=""; else K=1; L=50000000; S="_cfg4"; fi
    rm -rf gpurun_out/pmc
    KIND=$K LINES=$L PASSES="fetch write sq1 sq2" TP=200 bash tools/gpu_pmc.sh > $O/pmc_$w.log 2>&1 || { tail -20 $O/pmc_$w.log; exit 1; }
    KIND=$K LINES=$L python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_k_bwt$S.json || exit 1
    KIND=$K LINES=$L python3 tools/pmc_bwt_sq.py gpurun_out/pmc $O/pmc_k_bwt_sq$S.json || exit 1
    KIND=$K LINES=$L PMC_KERNELS="." python3 tools/pmc_bwt_sq.py gpurun_out/pmc $O/pmc_all_sq$S.json > /dev/null || exit 1
    mkdir -p $O/pmc_raw_$w && for p in fetch write sq1 sq2; do cp gpurun_out/pmc/$p/run_counter_collection.csv $O/pmc_raw_$w/$p.csv 2>/dev/null; done
  done
  ls $O
  exit 0
fi
timeout -k 10 600 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -20 $O/bench_cfg2.err; exit 1; }
cat $O/bench_cfg2.json
timeout -k 10 600 python bench.py --kind 1 --lines 50000000 --no-cpu-baseline --no-e2e > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -20 $O/bench_cfg4.err; exit 1; }
timeout -k 10 300 python bench.py --lines 12500000 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_eighth.json 2> $O/bench_eighth.err || { tail -20 $O/bench_eighth.err; exit 1; }
timeout -k 10 120 python tools/small_cost.py 300 > $O/cfg1_small_cost.json 2> $O/cfg1_small_cost.err || { tail -20 $O/cfg1_small_cost.err; exit 1; }
if [ -n "${CFG5:-}" ]; then
  timeout -k 10 900 python bench.py --kind 2 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
fi
BENCH_ARGS="--steps 2 --warmup 1" TP=300 bash tools/gpu_prof.sh > /dev/null || exit 1
cp gpurun_out/prof/run_kernel_stats.csv $O/cfg2_kernel_stats.csv
BENCH_ARGS="--steps 2 --warmup 1 --kind 1 --lines 50000000" TP=300 bash tools/gpu_prof.sh > /dev/null || exit 1
cp gpurun_out/prof/run_kernel_stats.csv $O/cfg4_kernel_stats.csv
python3 tools/kstats.py $O/cfg2_kernel_stats.csv 3 12
