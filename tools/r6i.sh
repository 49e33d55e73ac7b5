#!/bin/bash
# round-6 dev: mlp1 with 8-wave workgroups -- DIN GPU tests, kernel-stat A/B against 4 waves
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6i; mkdir -p $o
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_rank_pipeline.py tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
bash tools/din_ab.sh r6i prod nw4 prod nw4
