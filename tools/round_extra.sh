#!/bin/bash
# End-of-round evidence, second call (dev tool): busy-counter passes, the
# fused config-5 run (one rank's share) and the 8-shard config-4 replay.
# usage: tools/round_extra.sh TAG
set -o pipefail
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
bash tools/pmc_busy.sh $TAG/busy > gpurun_out/$TAG/busy.log 2>&1 || { tail -20 gpurun_out/$TAG/busy.log; exit 1; }
tail -3 gpurun_out/$TAG/busy.log
timeout -k 10 300 python -u bench.py --fused --fused-users 1250000 --no-cpu-baseline > gpurun_out/$TAG/fused.log 2>&1 || { tail -20 gpurun_out/$TAG/fused.log; exit 1; }
tail -1 gpurun_out/$TAG/fused.log | cut -c1-300
timeout -k 10 300 python3 tools/catalog_replay.py 8 > gpurun_out/$TAG/replay.log 2>&1 || { tail -20 gpurun_out/$TAG/replay.log; exit 1; }
tail -3 gpurun_out/$TAG/replay.log
echo extra-done
