#!/usr/bin/env bash
# GPU box: PMC passes (PASSES: sq1 sq2 fetch write) over an arbitrary python
# command (CMD, relative to the repo), one rocprofv3 run per pass, each under
# its own time limit.  Output: gpurun_out/pmcx/<pass>/
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/pmcx
cd /tmp && export TMPDIR=/tmp
for p in ${PASSES:-sq1 sq2}; do
  case $p in
    sq1) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" ;;
    sq2) C="SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS" ;;
    fetch) C="FETCH_SIZE" ;;
    write) C="WRITE_SIZE" ;;
    *) continue ;;
  esac
  timeout -s KILL ${TPMC:-150} rocprofv3 --kernel-trace --pmc $C -d $ROOT/gpurun_out/pmcx/$p -o run --output-format csv -- \
      python3 $ROOT/$CMD > $ROOT/gpurun_out/pmcx/$p.log 2>&1 || { echo "pmc pass $p failed"; tail -5 $ROOT/gpurun_out/pmcx/$p.log; exit 1; }
done
