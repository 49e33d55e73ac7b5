#!/bin/bash
# round-6 dev A/B: the D = 128 scan with 4 / 6 / 8 blocks per tile
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6g; mkdir -p $o
for v in prod tb6 tb8 prod tb8; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 300 python3 tools/scan128.py 250000 > $o/scan128_$v.txt 2>&1 || { tail $o/scan128_$v.txt; exit 1; }
  echo "== $v: $(tail -1 $o/scan128_$v.txt)"
done
