#!/bin/bash
# MFMA-busy / VALU-busy / stall counters for the dominant kernels (dev tool):
# separate rocprofv3 --pmc passes (8 SQ + 1 GRBM each) over the recall
# screen/finish driver, one DIN config-3 pass and the calibration loops
# (tools/calib/calib, built by __graft_entry__.build()), summarised by
# tools/pmc_busy.py.  usage: tools/pmc_busy.sh TAG
set -o pipefail
TAG=${1:-busy}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
S2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for set in "$S1" "$S2"; do
  i=$((i+1))
  REPS=1 timeout -s KILL 120 rocprofv3 --pmc $set -d $O/scr$i -o run --output-format csv -- python3 tools/prof_screen.py > $O/scr$i.log 2>&1 || { tail -5 $O/scr$i.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/din$i -o run --output-format csv -- python3 tools/din_prof.py 1 > $O/din$i.log 2>&1 || { tail -5 $O/din$i.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $set -d $O/cal$i -o run --output-format csv -- ./tools/calib/calib > $O/cal$i.log 2>&1 || { tail -5 $O/cal$i.log; exit 1; }
done
cat $O/cal1.log
python3 tools/pmc_busy.py $O > $O/busy.json && cat $O/busy.json
