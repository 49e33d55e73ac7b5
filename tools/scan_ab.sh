#!/bin/bash
# A/B the scan variants (NRK_SCAN_VARIANT) on config 2 (dev tool, GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_recall.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ${VARIANTS:-0 1 2 3}; do
  NRK_SCAN_VARIANT=$v timeout -k 10 120 python3 tools/screen_time.py 2>&1 | tail -1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/screen_time.py > $O/tool.log 2>&1 || { tail -30 $O/tool.log; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 6
