#!/usr/bin/env bash
# GPU box: selected GPU test files (TESTS, default all of tests/), one pytest
# process under its own time limit; log in gpurun_out/tests_<TAG>.log
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-sel}
timeout -k 10 ${TT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -15 gpurun_out/tests_$TAG.log
exit $rc
