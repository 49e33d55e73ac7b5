#!/bin/bash
# dev: context-feature + fused GPU tests, then the config-5 fused kernel stats
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_ctxfeat.py tests/test_gpu_fused.py -m gpu -q -x --timeout 150 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log
[ $rc -ne 0 ] && exit $rc
tools/prof_fused.sh $1
