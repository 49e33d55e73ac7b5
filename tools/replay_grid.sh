#!/bin/bash
# dev: config-4 one-GPU replays of several rank layouts (N or RxC) on one box.
# usage: tools/replay_grid.sh TAG layout...   e.g. tools/replay_grid.sh r6g 8 2x4 4x2
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
for n in "$@"; do
  timeout -k 10 300 python3 tools/catalog_replay.py $n > $o/replay_$n.txt 2>&1 || { tail $o/replay_$n.txt; exit 1; }
  echo "== $n: $(grep -h 'max per-rank\|owner rows' $o/replay_$n.txt | tr '\n' ' ')"
done
