#!/bin/bash
# DIN att_h A/B (dev tool, GPU box): DIN parity tests on the default build,
# pass times for NRK_DIN_ATT variants, per-kernel stats of the default.
# usage: tools/din_ab.sh TAG
set -o pipefail
TAG=${1:-dab}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_plugins.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in ${VARIANTS:-0 1}; do
    echo -n "att=$v "; NRK_DIN_ATT=$v timeout -k 10 120 python3 tools/din_time.py 10 2>&1 | tail -1 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/din_prof.py 3 > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 12
