#!/bin/bash
# dev: tools/scan_only.py per build on one box (prod = the in-tree library,
# otherwise news-recommendation-tc_amd/build_<v>/libnrk.so); a leading '+' on a
# variant name adds the 256-user oracle check.  usage: tools/scan_ab.sh TAG v...
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
for v in "$@"; do
  chk=""; [ "${v:0:1}" = "+" ] && { chk=--check; v=${v:1}; }
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 180 python3 tools/scan_only.py $chk > $o/so_$v.txt 2>&1 || { tail $o/so_$v.txt; exit 1; }
  echo "== $v: $(grep -h 'scan only\|oracle' $o/so_$v.txt | tr '\n' ' ')"
done
