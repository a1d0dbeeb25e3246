#!/usr/bin/env bash
# GPU box, end-of-round measurement package at the current sources (round 6),
# one PHASE per gpurun call:
#   PHASE=tests  every GPU test and smoke()
#   PHASE=pmc    stamped counters (FETCH/WRITE_SIZE traffic, SQ wait/issue
#                split) of the block sort for cfg2 and cfg4, of the transform
#                kernels (k_tf_*) for cfg2, and of every kernel (SQ) for cfg2
#   PHASE=pmc5   the same for cfg5 (block sort, transform, every kernel)
#   PHASE=pmc5nd the same for cfg5 with block reuse off (STARCH_DEDUPE=0)
#                (copy pmc_k_*.json to profiles/ before PHASE=bench: the bench
#                line attaches them only when their stamp matches)
#   PHASE=bench  the cfg2 bench line (CPU baseline, e2e, streamed, CLI, hpp,
#                bzlib legs), cfg4, 1/8 of cfg2, cfg1 fixed cost, cfg5 with and
#                without block reuse, and the rocprofv3 kernel-trace summaries
#                of cfg2 and cfg4
# Each GPU step has its own time limit; a failure ends the run.
set -o pipefail
mkdir -p gpurun_out/final
export PYTHONUNBUFFERED=1
O=gpurun_out/final
pmc() {   # workload suffix kind lines
  local w=$1 S=$2 K=$3 L=$4
  rm -rf gpurun_out/pmc
  KIND=$K LINES=$L PASSES="fetch write sq1 sq2" TP=${TP:-200} bash tools/gpu_pmc.sh > $O/pmc_$w.log 2>&1 || { tail -20 $O/pmc_$w.log; return 1; }
  KIND=$K LINES=$L python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_k_bwt$S.json || return 1
  KIND=$K LINES=$L python3 tools/pmc_bwt_sq.py gpurun_out/pmc $O/pmc_k_bwt_sq$S.json || return 1
  KIND=$K LINES=$L PMC_KERNELS="k_tf_" python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_k_tf$S.json || return 1
  KIND=$K LINES=$L PMC_KERNELS="." python3 tools/pmc_bwt_sq.py gpurun_out/pmc $O/pmc_all_sq$S.json > /dev/null || return 1
  KIND=$K LINES=$L PMC_KERNELS="." python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_all$S.json > /dev/null || return 1
  python3 tools/pmc_kernel_summary.py 'k_tf_fused|k_tf_place' gpurun_out/pmc > $O/pmc_tf_sq$S.txt || return 1
  rm -rf gpurun_out/pmc
}
case "${PHASE:-tests}" in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
      || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  cat $O/smoke.log
  ;;
pmc)
  pmc cfg2 "" 0 100000000 || exit 1
  pmc cfg4 _cfg4 1 50000000 || exit 1
  ls $O
  ;;
pmc5)
  TP=300 pmc cfg5 _cfg5 2 0 || exit 1
  ls $O
  ;;
pmc5nd)   # cfg5 with block reuse off: every block's doubling rounds
  export STARCH_DEDUPE=0
  TP=600 pmc cfg5nd _cfg5_nodedupe 2 0 || exit 1
  ls $O
  ;;
bench)
  timeout -k 10 600 python bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -20 $O/bench_cfg2.err; exit 1; }
  cat $O/bench_cfg2.json
  timeout -k 10 600 python bench.py --kind 1 --lines 50000000 --no-cpu-baseline --no-e2e > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -20 $O/bench_cfg4.err; exit 1; }
  timeout -k 10 300 python bench.py --lines 12500000 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_eighth.json 2> $O/bench_eighth.err || { tail -20 $O/bench_eighth.err; exit 1; }
  timeout -k 10 120 python tools/small_cost.py 300 > $O/cfg1_small_cost.json 2> $O/cfg1_small_cost.err || { tail -20 $O/cfg1_small_cost.err; exit 1; }
  timeout -k 10 600 python bench.py --kind 2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
  STARCH_DEDUPE=0 timeout -k 10 900 python bench.py --kind 2 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_cfg5_nodedupe.json 2> $O/bench_cfg5_nodedupe.err || { tail -20 $O/bench_cfg5_nodedupe.err; exit 1; }
  BENCH_ARGS="--steps 2 --warmup 1" TP=300 bash tools/gpu_prof.sh > /dev/null || exit 1
  cp gpurun_out/prof/run_kernel_stats.csv $O/cfg2_kernel_stats.csv
  BENCH_ARGS="--steps 2 --warmup 1 --kind 1 --lines 50000000" TP=300 bash tools/gpu_prof.sh > /dev/null || exit 1
  cp gpurun_out/prof/run_kernel_stats.csv $O/cfg4_kernel_stats.csv
  rm -rf gpurun_out/prof
  python3 tools/kstats.py $O/cfg2_kernel_stats.csv 3 12
  ;;
esac
