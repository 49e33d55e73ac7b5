#!/bin/bash
# round-6 dev: dim-128 scan ring slots 3 (product) vs 4 -- tools/scan128.py A/B
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6t; mkdir -p $o
set -o pipefail
for rep in 1 2; do
  for v in prod nsl4; do
    lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
    NRK_LIB_PATH=$lib timeout -k 10 300 python3 tools/scan128.py 250000 > $o/s128_${v}_$rep.log 2>&1 || { tail $o/s128_${v}_$rep.log; exit 1; }
    echo "== $v $rep: $(tail -1 $o/s128_${v}_$rep.log)"
  done
done
