#!/bin/bash
# round-6 dev: recall GPU tests on the two-round refine prefilter, bench A/B
# against the one-round build, D = 128 tile variants
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6e; mkdir -p $o
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_recall.py tests/test_gpu_embsim.py -x -q --timeout 150 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for rep in 1 2; do
  for v in prod pfd1; do
    lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
    NRK_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-din --no-itemcf --no-plugins > $o/bench_${v}_$rep.json 2> $o/bench_${v}_$rep.err || { tail $o/bench_${v}_$rep.err; exit 1; }
    echo "== $v $rep: $(grep -o '"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}' $o/bench_${v}_$rep.json | tr '\n' ' ')"
  done
done
for v in prod tb2 tb4; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 300 python3 tools/scan128.py 250000 > $o/scan128_$v.txt 2>&1 || { tail $o/scan128_$v.txt; exit 1; }
  echo "== $v: $(tail -1 $o/scan128_$v.txt)"
done
