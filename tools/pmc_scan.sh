#!/bin/bash
# dev: SQ counters of the config-2 scan (tools/scan_only.py) for one build,
# one rocprofv3 --pmc pass per counter set; summary via tools/pmc_sum.py.
# usage: tools/pmc_scan.sh TAG v "CTR CTR ..."
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; v=$2; mkdir -p $o
lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=$GRAFT_REPO_ROOT/news-recommendation-tc_amd/build_$v/libnrk.so
NRK_LIB_PATH=$lib timeout -s KILL 240 rocprofv3 --pmc $3 --output-format csv -d $o/pmc_$v -o run -- python3 tools/scan_only.py > $o/pmc_$v.log 2>&1 || { tail $o/pmc_$v.log; exit 1; }
python3 tools/pmc_sum.py $o/pmc_$v scan
