#!/bin/bash
# dev iteration: DIN GPU tests, then the config-3 DIN pass kernel stats
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_plugins.py -m gpu -q -x --timeout 150 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -3 $o/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/dprof -o run -- python3 tools/din_prof.py 10 > $o/din.txt 2>&1
rc=$?; tail -1 $o/din.txt; python3 tools/kstats.py $o/dprof/run_kernel_stats.csv 12
exit $rc
