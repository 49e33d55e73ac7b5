#!/bin/bash
# round-6 dev: resident-only persistent grids (select / shard band: 6 workgroups per CU; tower: occupancy-API grid)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6j; mkdir -p $o
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_recall.py -x -q --timeout 150 --timeout-method thread -k "not full_size" > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for rep in 1 2; do
  for v in prod g8 tg; do
    lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
    NRK_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-din --no-itemcf --no-plugins > $o/bench_${v}_$rep.json 2> $o/bench_${v}_$rep.err || { tail $o/bench_${v}_$rep.err; exit 1; }
    echo "== $v $rep: $(grep -o '"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}' $o/bench_${v}_$rep.json | tr '\n' ' ')"
  done
done
for v in prod g8; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 300 python3 tools/catalog_replay.py 8 > $o/replay_$v.txt 2>&1 || { tail $o/replay_$v.txt; exit 1; }
  echo "== replay $v: $(grep -h 'max per-rank\|owner rows' $o/replay_$v.txt | tr '\n' ' ')"
done
