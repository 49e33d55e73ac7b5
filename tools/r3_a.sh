#!/bin/bash
# Round-3 evidence, part A (GPU box): the full GPU suite, the near-tie counts
# of the full-size ItemCF tests, the default bench and its rocprofv3 kernel
# summary.  usage: tools/r3_a.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3a}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_gpu.log | head; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_itemcf.py -k full_size -q -s --timeout 280 --timeout-method thread > $O/itemcf_neartie.log 2>&1 || { tail -20 $O/itemcf_neartie.log; exit 1; }
grep "near-tie" $O/itemcf_neartie.log
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_under_rocprof.log 2>&1 || { tail -30 $O/bench_under_rocprof.log; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 14
