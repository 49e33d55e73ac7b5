#!/bin/bash
# dev: per build (prod or build_<name>): config-2 screen phases (HIP events)
# and the 8-shard config-4 replay, one box
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
for v in "$@"; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 200 python3 tools/scan_diag.py > $o/scan_$v.txt 2>&1 || exit 1
  NRK_LIB_PATH=$lib timeout -k 10 300 python3 tools/catalog_replay.py 8 > $o/replay_$v.log 2>&1 || exit 1
  echo "== $v: $(grep 'scan / select' $o/scan_$v.txt) | $(grep 'appends per user' $o/scan_$v.txt | cut -c1-60)"
  grep -E "shard 0 appended|max per-rank|owner rows" $o/replay_$v.log
done
