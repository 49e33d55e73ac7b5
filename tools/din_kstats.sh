#!/bin/bash
# per-kernel times of two DIN config-3 passes (dev tool). usage: tools/din_kstats.sh TAG
set -o pipefail
TAG=${1:-dk}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- python3 tools/din_prof.py 3 > gpurun_out/$TAG/log 2>&1 || { tail -20 gpurun_out/$TAG/log; exit 1; }
python3 tools/kstats.py gpurun_out/$TAG/prof/run_kernel_stats.csv 12
