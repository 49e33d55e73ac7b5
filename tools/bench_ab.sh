#!/bin/bash
# dev: the default recall bench (no DIN, no CPU baseline) per build, one box
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
i=0
for v in "$@"; do
  i=$((i+1))
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --no-din --no-cpu-baseline > $o/bench_${i}_$v.log 2>&1 || { tail $o/bench_${i}_$v.log; exit 1; }
  echo "== $v: $(tail -1 $o/bench_${i}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["ms_per_step"], d["phase_ms"])')"
done
