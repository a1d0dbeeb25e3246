#!/usr/bin/env bash
# GPU box: GPU tests, the concurrent-context probe (tools/lanes_probe.py) and
# SQ counters of every kernel over one cfg2 step (gpurun_out/pmc_all.json).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "${NOTESTS:-}" ]; then
  timeout -k 10 1000 python -u -m pytest -x -q -m gpu tests --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
  tail -2 gpurun_out/t_all.log
fi
timeout -k 10 300 python tools/lanes_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PASSES="sq1 sq2" LINES=100000000 TP=150 bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 1; }
PMC_KERNELS="." python3 tools/pmc_bwt_sq.py gpurun_out/pmc gpurun_out/pmc_all.json > /dev/null || exit 1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/pmc_all.json"))
for k, v in list(d["per_kernel"].items())[:24]:
    print("%-44s waitany %.2f waitinst %.2f active %.2f valu %.2f  insts valu %.3g lds %.3g bankc %.3g" % (
        k[:44], v["wait_any_frac"], v["wait_inst_any_frac"], v["active_inst_any_frac"], v["active_valu_frac"],
        v["insts_valu"], v["insts_lds"], v["lds_bank_conflict"]))
PY
