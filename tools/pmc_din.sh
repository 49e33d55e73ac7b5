#!/bin/bash
# PMC passes over one DIN pass (dev tool). usage: tools/pmc_din.sh TAG
set -o pipefail
TAG=${1:-pmcdin}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/$TAG/p$i -o run --output-format csv -- python3 tools/din_prof.py > gpurun_out/$TAG/p$i.log 2>&1 || { tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done
echo ok
