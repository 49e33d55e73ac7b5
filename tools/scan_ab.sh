#!/bin/bash
# dev: config-2 screen (tools/scan_diag.py) under each build: prod or build_<name>
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
for v in "$@"; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/s_$v -o run -- python3 tools/scan_diag.py > $o/scan_$v.txt 2>&1 || exit 1
  echo "== screen $v"; tail -3 $o/scan_$v.txt; python3 tools/kstats.py $o/s_$v/run_kernel_stats.csv 5
done
