#!/bin/bash
# Quick GPU check (dev tool): selected GPU tests, then a bench run (extra
# bench flags after --) under rocprofv3 --kernel-trace --stats.
# usage: tools/gpu_quick.sh TAG "test-files..." [bench flags...]
set -o pipefail
TAG=${1:-q}; TESTS=$2; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline "$@" > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep -v '^{' $O/bench.log | tail -8
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 25
