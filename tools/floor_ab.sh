#!/bin/bash
# dev: scan-only timing of the product build and the floor builds (build_fl*)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
for v in "$@"; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 120 python3 tools/scan_only.py > $o/so_$v.txt 2>&1 || { tail $o/so_$v.txt; exit 1; }
  echo "== $v: $(grep 'scan only' $o/so_$v.txt)"
done
