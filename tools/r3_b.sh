#!/bin/bash
# Round-3 evidence, part B (GPU box): FETCH_SIZE / WRITE_SIZE passes behind
# roofline.traffic, the SQ busy passes (+ the calibration loops), and the
# full-size EmbeddingSimilarity timing.  usage: tools/r3_b.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3b}; mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d $O/rec_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-din --no-cpu-baseline --no-plugins --no-itemcf > $O/rec_$c.log 2>&1 || { tail -5 $O/rec_$c.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc $c -d $O/din_$c -o run --output-format csv -- python3 tools/din_prof.py 2 > $O/din_$c.log 2>&1 || { tail -5 $O/din_$c.log; exit 1; }
done
echo traffic-done
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
S2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for set in "$S1" "$S2"; do
  i=$((i+1))
  REPS=1 timeout -s KILL 150 rocprofv3 --pmc $set -d $O/busy/scr$i -o run --output-format csv -- python3 tools/prof_screen.py > $O/scr$i.log 2>&1 || { tail -5 $O/scr$i.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $set -d $O/busy/din$i -o run --output-format csv -- python3 tools/din_prof.py 1 > $O/din$i.log 2>&1 || { tail -5 $O/din$i.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $set -d $O/busy/cal$i -o run --output-format csv -- ./tools/calib/calib > $O/cal$i.log 2>&1 || { tail -5 $O/cal$i.log; exit 1; }
done
grep -E "loop" $O/cal1.log | tail -2
./tools/calib/calib | tail -2
echo busy-done
timeout -k 10 300 python3 tools/embsim_bench.py > $O/embsim_fullsize.log 2>&1 || { tail -10 $O/embsim_fullsize.log; exit 1; }
tail -5 $O/embsim_fullsize.log
