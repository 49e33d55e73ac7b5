#!/bin/bash
# dev: recall GPU tests, then screen A/B ($2: comma list) and DIN A/B ($3: comma list)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_recall.py tests/test_gpu_din.py -m gpu -q -x --timeout 150 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log
[ $rc -ne 0 ] && exit $rc
tools/scan_ab.sh $1 ${2//,/ } || exit 1
[ -n "$3" ] && tools/din_ab.sh $1 ${3//,/ }
