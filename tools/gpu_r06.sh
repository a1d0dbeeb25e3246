#!/usr/bin/env bash
# GPU box (round 6 dev): cfg2 bench line (verified 24/24) + optional kernel
# trace summaries under variant environments.
#   VARIANTS="base KMAT=1"  each: rocprofv3 --kernel-trace --stats of a 2-step
#                           cfg2 bench under that env, summary -> gpurun_out/r06/<name>.txt
#   CFG4=1                  also the cfg4 bench line
#   EIGHTH=1                also the 1/8-of-cfg2 line
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r06
mkdir -p $O
export PYTHONUNBUFFERED=1
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $O/tests.log 2>&1 \
      || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e ${BENCH_EXTRA:-} > $O/cfg2.json 2> $O/cfg2.err || { tail -20 $O/cfg2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cfg2.json'));print('cfg2', d['ms_per_step'], d['value'], d['verify']['match'], d['stage_ms'])"
fi
if [ "${CFG4:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --kind 1 --lines 50000000 --no-cpu-baseline --no-e2e ${BENCH_EXTRA:-} > $O/cfg4.json 2> $O/cfg4.err || { tail -20 $O/cfg4.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cfg4.json'));print('cfg4', d['ms_per_step'], d['value'], d['verify']['match'], d['stage_ms'])"
fi
if [ "${EIGHTH:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --lines 12500000 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/eighth.json 2> $O/eighth.err || { tail -20 $O/eighth.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/eighth.json'));print('eighth', d['ms_per_step'], d['stage_ms'])"
fi
for v in ${VARIANTS:-}; do
  name=${v//=/_}
  rm -rf $O/prof_$name
  ( cd /tmp && export TMPDIR=/tmp && export STARCH_DEV_LANES=${STARCH_DEV_LANES:-1} && if [ "$v" != base ]; then export STARCH_$v; fi
    timeout -k 10 ${TP:-300} rocprofv3 --kernel-trace --stats -d $O/prof_$name -o run --output-format csv -- \
      python3 $ROOT/bench.py --steps 2 --warmup 1 ${PROF_ARGS:-} --no-cpu-baseline --no-e2e > $O/prof_$name.log 2>&1 ) \
      || { tail -20 $O/prof_$name.log; exit 1; }
  f=$(find $O/prof_$name -name '*kernel_stats.csv' | head -1)
  python3 $ROOT/tools/kstats.py "$f" 3 40 > $O/$name.txt
  tail -1 $O/prof_$name.log | cut -c1-300
  head -12 $O/$name.txt
done
for l in ${LIBS:-}; do
  STARCH_AMD_LIB=$ROOT/starch_amd/_sweep/$l/libstarch_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e ${BENCH_EXTRA:-} > $O/lib_$l.json 2> $O/lib_$l.err || { tail -20 $O/lib_$l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/lib_$l.json'));print('lib $l', d['ms_per_step'], d['value'], d['verify']['match'], d['stage_ms'])"
done
