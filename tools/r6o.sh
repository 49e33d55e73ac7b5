#!/bin/bash
# round-6 dev: the dim-128 finish's kernels (rocprofv3 kernel trace of tools/scan128.py)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6o; mkdir -p $o
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 tools/scan128.py 250000 > $o/prof.log 2>&1 || { tail $o/prof.log; exit 1; }
