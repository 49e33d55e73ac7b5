#!/bin/bash
# round-6 dev: config 5 (one rank's share) on the current tree + the recall GPU tests
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6u; mkdir -p $o
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_recall.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 300 python -u bench.py --fused --fused-users 1250000 --no-cpu-baseline > $o/fused.log 2>&1 || { tail -20 $o/fused.log; exit 1; }
tail -1 $o/fused.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}\|"frac": [0-9.]*' | tr '\n' ' '; echo
