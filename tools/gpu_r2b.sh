set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_recall.py tests/test_gpu_embsim.py tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/catalog_replay.py 8 > $O/replay.log 2>&1 || { tail -30 $O/replay.log; exit 1; }
cat $O/replay.log
timeout -k 10 300 python -u bench.py --no-din --no-itemcf --no-cpu-baseline > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-700
