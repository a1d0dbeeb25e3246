#!/usr/bin/env bash
# GPU box: the -m gpu suite, then (TRACE=1) a one-lane cfg2 kernel trace summary
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/t/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/t/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
if [ "${TRACE:-1}" = 1 ]; then
  BENCH=0 VARIANTS="base" bash tools/gpu_r06.sh > /dev/null || exit 1
  head -${TOPN:-40} gpurun_out/r06/base.txt
fi
