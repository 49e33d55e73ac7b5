#!/bin/bash
# round-6 dev: what bounds cf_pairs_flat_kernel -- kernel times of the product build, a no-atomic and a no-weight-math build
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6l; mkdir -p $o
set -o pipefail
for v in prod cfna cfnm; do
  lib=$PWD/news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=$PWD/news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_$v -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-din --no-plugins > $o/prof_$v.log 2>&1 || { tail $o/prof_$v.log; exit 1; }
done
