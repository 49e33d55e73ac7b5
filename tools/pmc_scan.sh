#!/bin/bash
# Busy / stall counters of the recall screen for the NRK_SCAN_VARIANT list in
# $VARIANTS (dev tool, GPU box): two rocprofv3 --pmc passes per variant over
# tools/prof_screen.py, summarised by tools/pmc_busy.py.  usage: pmc_scan.sh TAG
set -o pipefail
TAG=${1:-pmcscan}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
S2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for v in ${VARIANTS:-0}; do
  O=gpurun_out/$TAG/v$v
  mkdir -p $O
  i=0
  for set in "$S1" "$S2"; do
    i=$((i+1))
    NRK_SCAN_VARIANT=$v REPS=1 timeout -s KILL 120 rocprofv3 --pmc $set -d $O/scr$i -o run --output-format csv -- python3 tools/prof_screen.py > $O/scr$i.log 2>&1 || { tail -5 $O/scr$i.log; exit 1; }
  done
  echo "== variant $v"
  python3 tools/pmc_busy.py $O > $O/busy.json && cat $O/busy.json
done
