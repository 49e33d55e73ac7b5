#!/bin/bash
# round-6 dev: flat ItemCF pair kernel -- ItemCF GPU tests, bench ItemCF leg A/B against the per-user build, kernel stats
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6k; mkdir -p $o
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_itemcf.py -x -q --timeout 150 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for rep in 1 2; do
  for v in prod cfold; do
    lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
    NRK_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-din --no-plugins > $o/bench_${v}_$rep.json 2> $o/bench_${v}_$rep.err || { tail $o/bench_${v}_$rep.err; exit 1; }
    echo "== $v $rep: $(grep -o '"sim_ms": [0-9.]*\|"recall_ms": [0-9.]*' $o/bench_${v}_$rep.json | tr '\n' ' ')"
  done
done
for v in prod cfold; do
  lib=$PWD/news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=$PWD/news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_$v -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-din --no-plugins > $o/prof_$v.log 2>&1 || { tail $o/prof_$v.log; exit 1; }
done
