#!/bin/bash
# One GPU-box call: parity tests, bench, kernel-trace stats (dev tool).
# usage: tools/gpu_check.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-chk}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" \
  > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench.log 2>&1 || { tail -30 gpurun_out/$TAG/bench.log; exit 1; }
tail -1 gpurun_out/$TAG/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- \
  python3 bench.py --no-cpu-baseline > gpurun_out/$TAG/bench_prof.log 2>&1 || { tail -30 gpurun_out/$TAG/bench_prof.log; exit 1; }
echo done
