#!/bin/bash
# dev: tools/scan_only.py under rocprofv3 --kernel-trace --stats for one build
# (prod = the in-tree library); per-kernel summary via tools/kstats.py.
# usage: tools/prof_scan.sh TAG v
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; v=$2; mkdir -p $o
lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=$GRAFT_REPO_ROOT/news-recommendation-tc_amd/build_$v/libnrk.so
NRK_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$v -o run -- python3 tools/scan_only.py > $o/prof_$v.log 2>&1 || { tail $o/prof_$v.log; exit 1; }
python3 tools/kstats.py $o/prof_$v/run_kernel_stats.csv 14
