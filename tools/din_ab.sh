#!/bin/bash
# dev: config-3 DIN pass under each dev DIN build (kernel stats per variant)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=$1; case $o in gpurun_out/*) ;; *) o=gpurun_out/$o;; esac; shift; mkdir -p $o
for v in "$@"; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/$v -o run -- python3 tools/din_prof.py 10 > $o/$v.txt 2>&1 || exit 1
  echo "== $v: $(tail -1 $o/$v.txt)"; python3 tools/kstats.py $o/$v/run_kernel_stats.csv 3
done
