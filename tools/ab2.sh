#!/bin/bash
# A/B of scan variants on config 2 and the 8-shard replay (dev tool, GPU box).
# usage: VARIANTS="0 4" tools/ab2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab2}; mkdir -p $O
for v in ${VARIANTS:-0 4}; do
  NRK_SCAN_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_recall.py -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "variant $v: $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2; do
  for v in ${VARIANTS:-0 4}; do
    NRK_SCAN_VARIANT=$v timeout -k 10 120 python3 tools/screen_time.py 2>&1 | tail -1 || exit 1
  done
done
for v in ${VARIANTS:-0 4}; do
  echo "== replay, variant $v"
  NRK_SCAN_VARIANT=$v timeout -k 10 300 python3 tools/catalog_replay.py 8 > $O/replay_$v.log 2>&1 || { tail -20 $O/replay_$v.log; exit 1; }
  grep -E "appended|max per-rank|rank 0|owner rows" $O/replay_$v.log
done
