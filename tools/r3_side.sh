#!/bin/bash
# Side evidence on the current tree (dev tool): full-size EmbeddingSimilarity
# and the one-GPU 8-shard config-4 replay.  usage: tools/r3_side.sh TAG
set -o pipefail
TAG=${1:-side}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python3 -u tools/embsim_bench.py > $O/embsim_fullsize.log 2>&1 || { tail -20 $O/embsim_fullsize.log; exit 1; }
tail -4 $O/embsim_fullsize.log
timeout -k 10 300 python3 -u tools/catalog_replay.py 8 > $O/replay_8shards.log 2>&1 || { tail -20 $O/replay_8shards.log; exit 1; }
grep -E "appended|max per-rank|rank 0|owner rows|unsharded" $O/replay_8shards.log | head -12
