#!/usr/bin/env bash
# GPU box (dev): optional GPU tests (TESTS=1 all, TESTS=<-k expr>), then the cfg2
# bench line (verified 24/24 against the goldens) and the 1/8-of-cfg2 line
set -o pipefail
mkdir -p gpurun_out/chk
O=gpurun_out/chk
export PYTHONUNBUFFERED=1
if [ "${TESTS:-}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
elif [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$TESTS" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e ${BENCH_EXTRA:-} > $O/cfg2.json 2> $O/cfg2.err || { tail -20 $O/cfg2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg2.json'));print('cfg2', d['ms_per_step'], d['value'], d['verify']['match'], d['stage_ms'])"
timeout -k 10 300 python bench.py --lines 12500000 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e ${BENCH_EXTRA:-} > $O/eighth.json 2> $O/eighth.err || { tail -20 $O/eighth.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/eighth.json'));print('eighth', d['ms_per_step'], d['stage_ms'])"
