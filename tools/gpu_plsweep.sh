mkdir -p gpurun_out/r06
for v in plprof plprof_pu8 plprof_pu16; do
  STARCH_AMD_LIB=$PWD/starch_amd/_sweep/$v/libstarch_amd.so timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-verify 2> gpurun_out/r06/$v.err > gpurun_out/r06/$v.json || exit 1
  echo $v; grep plprof gpurun_out/r06/$v.err | tail -1
done
