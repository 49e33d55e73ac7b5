#!/bin/bash
# round-6 dev: user-tower workgroup size 512 (product) vs 1024 vs 256 (the previous) -- recall GPU tests, bench tower phase
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6y; mkdir -p $o
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_recall.py tests/test_gpu_plugins.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for rep in 1 2; do
  for v in prod tw1024 tw256; do
    lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
    NRK_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-din --no-itemcf --no-plugins > $o/bench_${v}_$rep.json 2> $o/bench_${v}_$rep.err || { tail $o/bench_${v}_$rep.err; exit 1; }
    echo "== $v $rep: $(grep -o '"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}' $o/bench_${v}_$rep.json | tr '\n' ' ')"
  done
done
