#!/bin/bash
# dev: recall GPU tests (product build), config-2 screen A/B over builds,
# phase stamps (build_sstamp) and the 8-shard config-4 replay
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_recall.py -m gpu -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log
[ $rc -ne 0 ] && exit $rc
tools/scan_ab.sh $(basename $o) "$@" || exit 1
grep -h "scan / select\|appends per user" $o/scan_*.txt
if [ -f news-recommendation-tc_amd/build_sstamp/libnrk.so ]; then
  NRK_LIB_PATH=news-recommendation-tc_amd/build_sstamp/libnrk.so timeout -k 10 200 python3 tools/scan_stamps.py > $o/stamps.txt 2>&1 || exit 1
  cat $o/stamps.txt
fi
timeout -k 10 400 python3 tools/catalog_replay.py 8 > $o/replay.log 2>&1 || { tail -20 $o/replay.log; exit 1; }
grep -E "appended|max per-rank|==" $o/replay.log
