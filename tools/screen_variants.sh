#!/bin/bash
# compare screen variants (dev tool). usage: tools/screen_variants.sh TAG v1 v2 ...
set -o pipefail
TAG=${1:-sv}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  NRK_SCREEN_VARIANT=$v timeout -k 10 200 python -u tools/screen_time.py > gpurun_out/$TAG/v$v.log 2>&1 || { tail -20 gpurun_out/$TAG/v$v.log; exit 1; }
  tail -1 gpurun_out/$TAG/v$v.log
done
