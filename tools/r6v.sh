#!/bin/bash
# round-6 dev: config 5 (one rank's share), dim-128 ring slots 4 (product) vs 3, one box
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6v; mkdir -p $o
set -o pipefail
for rep in 1 2; do
  for v in prod nsl3; do
    lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
    NRK_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --fused --fused-users 1250000 --no-cpu-baseline --steps 4 --warmup 1 > $o/fused_${v}_$rep.log 2>&1 || { tail -20 $o/fused_${v}_$rep.log; exit 1; }
    echo "== $v $rep: $(tail -1 $o/fused_${v}_$rep.log | grep -o '"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}' | tr '\n' ' ')"
  done
done
