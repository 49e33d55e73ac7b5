#!/bin/bash
# dev: kernel stats of the config-3 DIN pass and the screen variants (product, 16-KB tiles, two-pass F=8 / F=4)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/dprof -o run -- python3 tools/din_prof.py 10 > $o/din.txt 2>&1
tail -1 $o/din.txt; python3 tools/kstats.py $o/dprof/run_kernel_stats.csv 12
for v in "" _t16 8 4; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ -n "$v" ] && lib=news-recommendation-tc_amd/build_dev$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/s$v -o run -- python3 tools/scan_diag.py > $o/scan$v.txt 2>&1
  echo "== screen variant [$v]"; tail -3 $o/scan$v.txt; python3 tools/kstats.py $o/s$v/run_kernel_stats.csv 6
done
