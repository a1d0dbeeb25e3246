# GPU box: ByteP MTF (17..30 symbols, cfg4) with the zero runs from neighbour compares vs stored indices
mkdir -p gpurun_out/bs
timeout -k 10 600 python -u -m pytest tests/test_gpu_mtf.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bs/t.log 2>&1
rc=$?; tail -3 gpurun_out/bs/t.log; [ $rc -eq 0 ] || exit $rc
run() {  # name lib lanes args...
  local name=$1 lib=$2 L=$3; shift 3
  STARCH_AMD_LIB=$lib STARCH_DEV_LANES=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e "$@" > gpurun_out/bs/$name.json 2> gpurun_out/bs/$name.err || { tail gpurun_out/bs/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bs/$name.json'));print('$name', d['ms_per_step'], d['value'], d['verify']['all'], d['stage_ms'])"
}
B=starch_amd/_build
A="--kind 1 --lines 50000000 --steps 3 --warmup 1"
run cfg4_l1_new $B/libstarch_amd.so 1 $A
run cfg4_l1_six $B/v_six/libstarch_amd.so 1 $A
run cfg4_l2_new $B/libstarch_amd.so 2 $A
run cfg4_l2_six $B/v_six/libstarch_amd.so 2 $A
