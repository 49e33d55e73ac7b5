#!/bin/bash
# Round-3 dev loop (GPU box): selected GPU tests, then the config-2 screen /
# finish timing under rocprofv3 --kernel-trace --stats.
# usage: tools/gpu_r3.sh TAG "test-files..." [extra tool]
set -o pipefail
TAG=${1:-r3}; TESTS=$2; TOOL=${3:-tools/screen_time.py}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?
  grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -60
  [ $rc -eq 0 ] || { tail -60 $O/pytest.log; exit 1; }
fi
if [ "$TOOL" != "none" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $TOOL > $O/tool.log 2>&1 || { tail -30 $O/tool.log; exit 1; }
  tail -5 $O/tool.log
  python3 tools/kstats.py $O/prof/run_kernel_stats.csv 20
fi
