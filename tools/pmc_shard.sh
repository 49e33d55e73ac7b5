#!/bin/bash
# SQ / TCC counters of the shard-path kernels over the 8-shard replay (dev tool).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcsh}; mkdir -p $O
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
S2="FETCH_SIZE SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
i=0
for set in "$S1" "$S2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set -d $O/p$i -o run --output-format csv -- python3 tools/catalog_replay.py 8 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_sum.py $O "ip_shard|ip_scan|ip_refine|ip_select"
