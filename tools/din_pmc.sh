#!/bin/bash
# dev: DIN config-3 pass kernel stats + two PMC passes per build (prod or build_<name>)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
S2="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for v in "$@"; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$v -o run -- python3 tools/din_prof.py 10 > $o/$v.txt 2>&1 || exit 1
  echo "== $v: $(tail -1 $o/$v.txt)"; python3 tools/kstats.py $o/$v/run_kernel_stats.csv 4
  i=0
  for set in "$S1" "$S2"; do
    i=$((i+1))
    NRK_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc $set -d $o/${v}_pmc$i -o run --output-format csv -- python3 tools/din_prof.py 1 > $o/${v}_pmc$i.log 2>&1 || { tail -5 $o/${v}_pmc$i.log; exit 1; }
  done
  python3 tools/pmc_sum.py $o/${v}_pmc1 "din_att_tm|din_wh2" ; python3 tools/pmc_sum.py $o/${v}_pmc2 "din_att_tm|din_wh2"
done
