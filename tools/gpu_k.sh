#!/bin/bash
# Recall / embsim / plugin GPU tests + rehearsal + shard debug + A/B (dev tool)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-gk}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_recall.py tests/test_gpu_embsim.py tests/test_gpu_plugins.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/shard_debug.py 8 2>&1 | grep -v "amdgpu.ids" | cut -c1-200 || exit 1
tools/rehearse.sh $1_reh "2 3" || exit 1
VARIANTS="0" tools/ab2.sh $1_ab
