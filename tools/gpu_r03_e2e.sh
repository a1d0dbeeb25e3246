#!/usr/bin/env bash
# GPU box: the host-input paths -- stream/pipelined tests, then the e2e probe
# (tools/e2e_trace.py) under lane / batch-count variants (VARIANTS="L:B ...").
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py > gpurun_out/t_stream.log 2>&1 || { tail -40 gpurun_out/t_stream.log; exit 1; }
  tail -3 gpurun_out/t_stream.log
fi
for v in ${VARIANTS:-2:8}; do
  L=${v%%:*}; B=${v##*:}
  STARCH_TRACE=1 STARCH_LANES=$L STARCH_PIPE_BATCHES=$B timeout -k 10 200 python -u tools/e2e_trace.py > gpurun_out/e2e_$L_$B.log 2>&1 || { tail -30 gpurun_out/e2e_$L_$B.log; exit 1; }
  cp gpurun_out/e2e_$L_$B.log gpurun_out/e2e_${L}_${B}.log
  echo "lanes=$L batches=$B"; grep -v "^\[starch" gpurun_out/e2e_${L}_${B}.log | grep -v amdgpu.ids
done
