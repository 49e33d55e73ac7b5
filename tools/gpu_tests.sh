#!/bin/bash
# Selected GPU tests in one process (dev tool). usage: tools/gpu_tests.sh TAG test-files...
set -o pipefail
TAG=${1:-t}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -60 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
