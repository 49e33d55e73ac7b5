#!/bin/bash
# round-6 dev: DIN absmax with one atomic per workgroup -- DIN GPU tests, kernel times, bench DIN pass
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6z; mkdir -p $o
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_din.py tests/test_rank_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python3 tools/din_prof.py 2 > $o/prof.log 2>&1 || { tail $o/prof.log; exit 1; }
grep -h 'absmax' $o/prof/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-itemcf --no-plugins > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
grep -o '"ms_per_pass": [0-9.]*' $o/bench.json
