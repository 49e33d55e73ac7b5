#!/bin/bash
# dev: recall GPU tests on the product build, then the config-2 screen A/B
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_recall.py -m gpu -q -x --timeout 200 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log
[ $rc -ne 0 ] && exit $rc
tools/scan_ab.sh $(basename $o) "$@"
if [ -f news-recommendation-tc_amd/build_sstamp/libnrk.so ]; then
  NRK_LIB_PATH=news-recommendation-tc_amd/build_sstamp/libnrk.so timeout -k 10 200 python3 tools/scan_stamps.py > $o/stamps.txt 2>&1 || exit 1
  cat $o/stamps.txt
fi
