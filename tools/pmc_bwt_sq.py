#!/usr/bin/env python3
"""What limits the block sort, from rocprofv3 SQ counters (tools/gpu_pmc.sh
PASSES="sq1 sq2" over one cfg2 bench step), stamped with the kernel sources.

Per block-sort kernel (k3_*, k_fallback*, k_last_col) and summed over the
stage: wave cycles split into WAIT_ANY (wave parked on s_waitcnt / barrier:
memory latency), WAIT_INST_ANY (issue stall: dependency / pipe busy) and
ACTIVE_INST_ANY (issuing) -- disjoint, and about WAVE_CYCLES together
(MI355X_MICROARCH.md, rocprofv3 PMC slots) -- plus instruction mix and LDS
bank conflicts.  bench.py reads the stage summary as roofline.limiter when
the stamp matches its sources.
usage: pmc_bwt_sq.py [PMC_DIR] [OUT_JSON]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import src_stamp  # noqa: E402
from tools.pmc_bwt_traffic import is_bwt  # noqa: E402


KSEL = os.environ.get("PMC_KERNELS", "")     # regex over kernel names (default: the block-sort kernels)


def load(d):
    tot = collections.defaultdict(collections.Counter)
    for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if (re.search(KSEL, r["Kernel_Name"]) if KSEL else is_bwt(r["Kernel_Name"])):
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return tot


def derive(c):
    wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    return {
        "wave_cycles": c.get("SQ_WAVE_CYCLES", 0.0),
        "wait_any_frac": round(c.get("SQ_WAIT_ANY", 0.0) / wc, 4),
        "wait_inst_any_frac": round(c.get("SQ_WAIT_INST_ANY", 0.0) / wc, 4),
        "active_inst_any_frac": round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4),
        "active_valu_frac": round(c.get("SQ_ACTIVE_INST_VALU", 0.0) / wc, 4),
        "insts_valu": c.get("SQ_INSTS_VALU", 0.0), "insts_lds": c.get("SQ_INSTS_LDS", 0.0),
        "insts_salu": c.get("SQ_INSTS_SALU", 0.0), "insts_vmem_rd": c.get("SQ_INSTS_VMEM_RD", 0.0),
        "insts_vmem_wr": c.get("SQ_INSTS_VMEM_WR", 0.0), "lds_bank_conflict": c.get("SQ_LDS_BANK_CONFLICT", 0.0),
        "waves": c.get("SQ_WAVES", 0.0),
    }


def limiter(d):
    parts = {"memory latency (waves parked on s_waitcnt/barriers)": d["wait_any_frac"],
             "issue stalls (dependencies, busy pipes)": d["wait_inst_any_frac"],
             "instruction issue": d["active_inst_any_frac"]}
    return max(parts, key=parts.get)


def main():
    pmc = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_k_bwt_sq.json"
    a = load(os.path.join(pmc, "sq1"))
    b = load(os.path.join(pmc, "sq2"))
    per, total = {}, collections.Counter()
    for k in sorted(set(a) | set(b)):
        c = collections.Counter(a.get(k, {}))
        c.update(b.get(k, {}))
        total.update(c)
        per[k] = derive(c)
    stage = derive(total)
    res = {"src_stamp": src_stamp(), "lines": int(os.environ.get("LINES", "100000000")),
           "kind": int(os.environ.get("KIND", "0")),
        "block_reuse": os.environ.get("STARCH_DEDUPE") != "0",
           "method": "rocprofv3 --kernel-trace --pmc, passes sq1 (SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS "
                     "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES) and sq2 (SQ_BUSY_CYCLES "
                     "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU "
                     "SQ_INSTS_SMEM SQ_WAIT_INST_LDS) over one cfg2 bench step; block-sort kernels summed",
           "stage": stage, "limiter": limiter(stage),
           "per_kernel": dict(sorted(per.items(), key=lambda kv: -kv[1]["wave_cycles"]))}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({"limiter": res["limiter"], "stage": stage}))


if __name__ == "__main__":
    main()
