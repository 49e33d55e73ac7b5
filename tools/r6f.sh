#!/bin/bash
# round-6: recall / fused GPU tests on the 4-block dim-128 tiles, then the config-5 fused bench
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6f; mkdir -p $o
set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_recall.py tests/test_gpu_embsim.py tests/test_gpu_fused.py tests/test_capi.py -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 400 python -u bench.py --fused --fused-users 1250000 --no-cpu-baseline > $o/fused.log 2>&1 || { tail -20 $o/fused.log; exit 1; }
tail -1 $o/fused.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}\|"frac": [0-9.]*'
