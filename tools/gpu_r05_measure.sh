#!/usr/bin/env bash
# GPU box (round 5): the host-facing legs of cfg2 (e2e, streamed, CLI, the
# starch3api.hpp surface, BZ_RUN through the bzlib ABI), cfg5 with and without
# exact block reuse, and FETCH/WRITE counters of every kernel for cfg2 and cfg5
# (PMC_CFG2=1 / PMC_CFG5=1).  Each GPU step under its own limit; a failure ends it.
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
export PYTHONUNBUFFERED=1
if [ -z "${SKIP_CFG2:-}" ]; then
  timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -20 $O/bench_cfg2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_cfg2.json'));e=d['e2e'];print('cfg2',d['ms_per_step'],d['value'],d['verify']['match']);print(json.dumps({k:(v if not isinstance(v,dict) else {a:b for a,b in v.items() if a!='includes'}) for k,v in e.items() if k!='includes'}))"
fi
if [ -n "${CFG5:-}" ]; then
  timeout -k 10 600 python bench.py --kind 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -20 $O/bench_cfg5.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_cfg5.json'));print('cfg5',d['ms_per_step'],d['value'],d['verify']['match'],d['stage_ms'],d['bwt'])"
  STARCH_DEDUPE=0 timeout -k 10 900 python bench.py --kind 2 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_cfg5_nodedupe.json 2> $O/bench_cfg5_nodedupe.err || { tail -20 $O/bench_cfg5_nodedupe.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_cfg5_nodedupe.json'));print('cfg5-nodedupe',d['ms_per_step'],d['value'],d['verify']['match'],d['stage_ms'],d['bwt'])"
fi
if [ -n "${PMC_CFG2:-}" ]; then
  rm -rf gpurun_out/pmc
  KIND=0 LINES=100000000 PASSES="fetch write" TP=200 bash tools/gpu_pmc.sh > $O/pmc_cfg2.log 2>&1 || { tail -20 $O/pmc_cfg2.log; exit 1; }
  KIND=0 LINES=100000000 PMC_KERNELS="k_tf_" python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_k_tf.json || exit 1
  KIND=0 LINES=100000000 PMC_KERNELS="." python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_all_cfg2.json || exit 1
  KIND=0 LINES=100000000 python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_k_bwt.json || exit 1
fi
if [ -n "${PMC_CFG5:-}" ]; then
  rm -rf gpurun_out/pmc
  KIND=2 LINES=0 PASSES="fetch write sq1 sq2" TP=300 bash tools/gpu_pmc.sh > $O/pmc_cfg5.log 2>&1 || { tail -20 $O/pmc_cfg5.log; exit 1; }
  KIND=2 LINES=0 python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_k_bwt_cfg5.json || exit 1
  KIND=2 LINES=0 python3 tools/pmc_bwt_sq.py gpurun_out/pmc $O/pmc_k_bwt_sq_cfg5.json || exit 1
  KIND=2 LINES=0 PMC_KERNELS="k_tf_" python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_k_tf_cfg5.json || exit 1
  KIND=2 LINES=0 PMC_KERNELS="." python3 tools/pmc_bwt_traffic.py gpurun_out/pmc $O/pmc_all_cfg5.json || exit 1
fi
ls $O
