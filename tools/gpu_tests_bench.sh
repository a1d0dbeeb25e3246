mkdir -p gpurun_out/t
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/t/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/t/cfg2.json 2> gpurun_out/t/cfg2.err || { tail gpurun_out/t/cfg2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/t/cfg2.json'));print(d['ms_per_step'], d['value'], d['verify']['all'], d['stage_ms'])"
