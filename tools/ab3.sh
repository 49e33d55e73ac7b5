#!/bin/bash
# Round-3 A/B in one GPU call (dev tool): recall / DIN parity tests, DIN
# att_h variants (NRK_DIN_ATT), scan variants (NRK_SCAN_VARIANT), then
# per-kernel stats of a bench run.  usage: tools/ab3.sh TAG
set -o pipefail
TAG=${1:-ab3}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_recall.py tests/test_gpu_din.py tests/test_gpu_plugins.py} -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in ${DVARS:-0 1}; do
    echo -n "din=$v "; NRK_DIN_WH=$v timeout -k 10 120 python3 tools/din_time.py 10 2>&1 | tail -1 || exit 1
  done
  for v in ${SVARS:-0 6 7 8}; do
    NRK_SCAN_VARIANT=$v timeout -k 10 120 python3 tools/screen_time.py 2>&1 | tail -1 || exit 1
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-plugins --no-itemcf > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep -v '^{' $O/bench.log | tail -4
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 20
