#!/bin/bash
# round-6 dev A/B: recall bench (tower rows in flight 16 vs 8, alternating),
# then the D = 128 scan with 8-KB vs 16-KB tiles
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6c; mkdir -p $o
set -o pipefail
for rep in 1 2; do
  for v in prod tt8; do
    lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
    NRK_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-din --no-itemcf --no-plugins > $o/bench_${v}_$rep.json 2> $o/bench_${v}_$rep.err || { tail $o/bench_${v}_$rep.err; exit 1; }
    echo "== $v $rep: $(grep -o '"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}' $o/bench_${v}_$rep.json | tr '\n' ' ')"
  done
done
for v in prod tb2; do
  lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
  NRK_LIB_PATH=$lib timeout -k 10 300 python3 tools/scan128.py 250000 > $o/scan128_$v.txt 2>&1 || { tail $o/scan128_$v.txt; exit 1; }
  echo "== $v: $(tail -1 $o/scan128_$v.txt)"
done
