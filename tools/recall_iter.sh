#!/bin/bash
# dev: recall GPU tests, config-2 screen diagnostics + kernel stats, 8-shard replay
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_recall.py -m gpu -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log
[ $rc -ne 0 ] && exit $rc
tools/scan_ab.sh $1 prod || exit 1
timeout -k 10 400 python3 tools/catalog_replay.py 8 > $o/replay.log 2>&1 || { tail -20 $o/replay.log; exit 1; }
grep -E "appended|max per-rank|==" $o/replay.log
