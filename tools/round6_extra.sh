#!/bin/bash
# Round-6 evidence, part 2 (dev tool): busy-counter passes, one rank's share of
# config 5, the 8-shard config-4 replay, and the gloo rehearsal of the 2- and
# 3-rank bench.  usage: tools/round6_extra.sh TAG
set -o pipefail
TAG=${1:-r6x}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
bash tools/pmc_busy.sh $TAG/busy > $O/busy_run.log 2>&1 || { tail -20 $O/busy_run.log; exit 1; }
echo busy-done
timeout -k 10 300 python -u bench.py --fused --fused-users 1250000 --no-cpu-baseline > $O/fused.log 2>&1 || { tail -20 $O/fused.log; exit 1; }
tail -1 $O/fused.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}\|"frac": [0-9.]*' | tr '\n' ' '; echo
timeout -k 10 300 python3 tools/catalog_replay.py 8 > $O/replay_8.txt 2>&1 || { tail $O/replay_8.txt; exit 1; }
grep -h 'max per-rank\|owner rows' $O/replay_8.txt
bash tools/rehearse.sh $TAG/reh "2 3" > $O/reh.log 2>&1 || { tail -20 $O/reh.log; exit 1; }
echo extra-done
