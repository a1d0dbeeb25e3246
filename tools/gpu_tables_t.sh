# GPU box: k_tables32 workgroup size A/B (STARCH_TABLES_T) on cfg2 and 1/8 of cfg2, two lanes
mkdir -p gpurun_out/tt
run() {  # name env... -- args
  local name=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e "$@" > gpurun_out/tt/$name.json 2> gpurun_out/tt/$name.err || { tail gpurun_out/tt/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/tt/$name.json'));print('$name', d['ms_per_step'], d['value'], d['verify']['all'], d['stage_ms'])"
}
for T in 256 512 1024; do run cfg2_t$T STARCH_TABLES_T=$T --; done
for T in 1024 512; do run eighth_t$T STARCH_TABLES_T=$T -- --lines 12500000 --steps 10 --warmup 3; done
