# GPU box: parity subset, then cfg2 (one and two lanes) and cfg4
mkdir -p gpurun_out/u8
timeout -k 10 600 python -u -m pytest tests/test_gpu_mtf.py tests/test_gpu_parity.py tests/test_gpu_bwt.py tests/test_gpu_dedupe.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/u8/t.log 2>&1
rc=$?; tail -4 gpurun_out/u8/t.log; [ $rc -eq 0 ] || exit $rc
run() {  # name lib lanes args...
  local name=$1 lib=$2 L=$3; shift 3
  STARCH_AMD_LIB=$lib STARCH_DEV_LANES=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e "$@" > gpurun_out/u8/$name.json 2> gpurun_out/u8/$name.err || { tail gpurun_out/u8/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/u8/$name.json'));print('$name', d['ms_per_step'], d['value'], d['verify']['all'], d['stage_ms'])"
}
B=starch_amd/_build
for v in ${VARIANTS:-}; do run cfg2_l1_$v $B/$v/libstarch_amd.so 1; done
run cfg2_l1 $B/libstarch_amd.so 1
run cfg2_l2 $B/libstarch_amd.so 2
[ "${CFG4:-1}" = 1 ] && run cfg4 $B/libstarch_amd.so 2 --kind 1 --lines 50000000 --steps 5 --warmup 2
true
