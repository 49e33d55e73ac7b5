#!/bin/bash
# End-of-round evidence in one GPU-box call (dev tool): tools/round_profile.sh
# (GPU tests, bench, kernel stats, FETCH/WRITE passes), the busy-counter
# passes, and one rank's share of the fused config-5 pipeline.
# usage: tools/round_final.sh TAG
set -o pipefail
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/round_profile.sh $TAG || exit 1
bash tools/pmc_busy.sh $TAG/busy > /dev/null || exit 1
timeout -k 10 300 python -u bench.py --fused --fused-users 1250000 --no-cpu-baseline > gpurun_out/$TAG/fused.log 2>&1 || { tail -20 gpurun_out/$TAG/fused.log; exit 1; }
tail -1 gpurun_out/$TAG/fused.log | cut -c1-300
echo final-done
