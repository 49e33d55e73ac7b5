#!/bin/bash
# round-6 dev: band statistics at D = 128 (5M items) and D = 32 (config 2)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6q; mkdir -p $o
set -o pipefail
timeout -k 10 300 python3 tools/band_stats.py 128 100000 5000000 > $o/b128.log 2>&1 || { tail $o/b128.log; exit 1; }
timeout -k 10 300 python3 tools/band_stats.py 32 250000 364047 > $o/b32.log 2>&1 || { tail $o/b32.log; exit 1; }
cat $o/b128.log $o/b32.log
