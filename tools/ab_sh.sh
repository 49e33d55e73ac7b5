#!/bin/bash
# A/B of the persistent grid of the select / shard kernels (NRK_SH_WG) on the
# 8-shard replay, plus one rocprofv3 kernel summary (dev tool, GPU box).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-absh}; mkdir -p $O
for w in ${WGS:-4 8 16 32}; do
  echo "== NRK_SH_WG=$w"
  NRK_SH_WG=$w timeout -k 10 120 python3 tools/screen_time.py 2>&1 | tail -1 || exit 1
  NRK_SH_WG=$w timeout -k 10 300 python3 tools/catalog_replay.py 8 > $O/replay_$w.log 2>&1 || { tail -20 $O/replay_$w.log; exit 1; }
  grep -E "max per-rank|rank 0" $O/replay_$w.log
done
for d in ${DBGS:-}; do
  echo "== NRK_SH_DBG=$d"
  NRK_SH_DBG=$d timeout -k 10 300 python3 tools/catalog_replay.py 8 > $O/replay_d$d.log 2>&1 || { tail -20 $O/replay_d$d.log; exit 1; }
  grep -E "max per-rank|rank 0" $O/replay_d$d.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/catalog_replay.py 8 > $O/tool.log 2>&1 || { tail -30 $O/tool.log; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 8
