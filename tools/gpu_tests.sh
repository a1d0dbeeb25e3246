#!/usr/bin/env bash
# Run on the GPU box: GPU parity tests, each step under its own time limit.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${T1:-900} python -m pytest tests -m gpu ${XFLAG--x} -v ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
