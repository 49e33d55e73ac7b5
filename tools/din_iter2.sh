#!/bin/bash
# dev: DIN GPU tests, kernel stats of prod and the listed builds, phase stamps
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; shift; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_plugins.py -m gpu -q -x --timeout 150 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log
[ $rc -ne 0 ] && exit $rc
tools/din_ab.sh $o prod "$@" || exit 1
NRK_LIB_PATH=news-recommendation-tc_amd/build_stamp/libnrk.so timeout -k 10 200 python3 tools/din_stamps.py
