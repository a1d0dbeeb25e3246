#!/usr/bin/env bash
# GPU box (dev): bench cfg2 and 1/8 of cfg2 with each library variant under
# starch_amd/_sweep/<name>/ plus the in-tree build ("base"); one JSON per run
set -o pipefail
mkdir -p gpurun_out/sweep
for v in base $(ls starch_amd/_sweep 2>/dev/null); do
  if [ $v = base ]; then L=""; else L=starch_amd/_sweep/$v/libstarch_amd.so; fi
  STARCH_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-verify > gpurun_out/sweep/$v.json 2> gpurun_out/sweep/$v.err || { tail -5 gpurun_out/sweep/$v.err; exit 1; }
  STARCH_AMD_LIB=$L timeout -k 10 200 python bench.py --lines 12500000 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-verify > gpurun_out/sweep/${v}_8.json 2> gpurun_out/sweep/${v}_8.err || { tail -5 gpurun_out/sweep/${v}_8.err; exit 1; }
  python3 -c "
import json;a=json.load(open('gpurun_out/sweep/$v.json'));b=json.load(open('gpurun_out/sweep/${v}_8.json'))
print('%-10s cfg2 %.3f ms  tables %.3f  bwt %.3f | 1/8 %.3f ms tables %.3f' % ('$v', a['ms_per_step'], a['stage_ms']['ms_tables'], a['stage_ms']['ms_bwt'], b['ms_per_step'], b['stage_ms']['ms_tables']))"
done
