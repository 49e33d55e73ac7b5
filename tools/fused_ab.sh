#!/bin/bash
# dev: config-5 fused bench (one rank's share) per build, one box
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
for v in "$@"; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --fused --fused-users 1250000 --no-cpu-baseline --steps 5 --warmup 2 > $o/fused_$v.log 2>&1 || { tail $o/fused_$v.log; exit 1; }
  echo "== $v: $(tail -1 $o/fused_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["phase_ms"])')"
done
