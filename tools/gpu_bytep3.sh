# GPU box: three-word byte lists (17..24 symbols) and per-batch class launches: parity + cfg4 / cfg2 / 1/8
mkdir -p gpurun_out/b3
timeout -k 10 600 python -u -m pytest tests/test_gpu_mtf.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_dedupe.py tests/test_gpu_bzlib_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/b3/t.log 2>&1
rc=$?; tail -3 gpurun_out/b3/t.log; [ $rc -eq 0 ] || exit $rc
run() {  # name lanes args...
  local name=$1 L=$2; shift 2
  STARCH_DEV_LANES=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e "$@" > gpurun_out/b3/$name.json 2> gpurun_out/b3/$name.err || { tail gpurun_out/b3/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b3/$name.json'));print('$name', d['ms_per_step'], d['value'], d['verify']['all'], d['stage_ms'])"
}
run cfg4_l1 1 --kind 1 --lines 50000000 --steps 3 --warmup 1
run cfg4_l2 2 --kind 1 --lines 50000000 --steps 3 --warmup 1
run cfg2_l2 2
run eighth_l2 2 --lines 12500000 --steps 10 --warmup 3
