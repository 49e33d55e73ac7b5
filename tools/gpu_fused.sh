#!/bin/bash
# config-5 fused runs (dev tool). usage: tools/gpu_fused.sh TAG
set -o pipefail
TAG=${1:-fz}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u bench.py --fused --fused-users 100000 --fused-items 500000 --steps 2 --warmup 1 > $O/small.log 2>&1 || { tail -30 $O/small.log; exit 1; }
tail -1 $O/small.log | cut -c1-600
timeout -k 10 600 python -u bench.py --fused --fused-users 1250000 --no-cpu-baseline --steps 3 --warmup 1 > $O/config5_1rank.log 2>&1 || { tail -30 $O/config5_1rank.log; exit 1; }
tail -1 $O/config5_1rank.log | cut -c1-900
