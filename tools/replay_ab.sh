#!/bin/bash
# dev: tools/catalog_replay.py N per build on one box (prod = the in-tree
# library, otherwise news-recommendation-tc_amd/build_<v>/libnrk.so).
# usage: tools/replay_ab.sh TAG N v...
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; n=$2; shift 2; mkdir -p $o
for v in "$@"; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 240 python3 tools/catalog_replay.py $n > $o/replay_${n}_$v.txt 2>&1 || { tail $o/replay_${n}_$v.txt; exit 1; }
  echo "== $v: $(grep -h 'max per-rank\|owner rows\|shard 0 app' $o/replay_${n}_$v.txt | tr '\n' ' ')"
done
