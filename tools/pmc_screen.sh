#!/bin/bash
# PMC passes over the recall screen/finish (dev tool). usage: tools/pmc_screen.sh TAG
set -o pipefail
TAG=${1:-pmc}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
[ -f gpurun_out/$TAG/../counters.txt ] || timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  REPS=1 timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/$TAG/p$i -o run --output-format csv -- python3 tools/prof_screen.py > gpurun_out/$TAG/p$i.log 2>&1 || { tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done
echo ok
