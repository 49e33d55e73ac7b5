#!/bin/bash
# round-6 dev: dim-128 refine (ring-batched exact rounds, chunked exact dot) -- recall GPU tests, tools/scan128.py A/B
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6n; mkdir -p $o
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_recall.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
for rep in 1 2; do
  for v in prod rfold; do
    lib=news-recommendation-tc_amd/nrk/libnrk.so; [ "$v" != prod ] && lib=news-recommendation-tc_amd/build_$v/libnrk.so
    NRK_LIB_PATH=$lib timeout -k 10 300 python3 tools/scan128.py 250000 > $o/s128_${v}_$rep.log 2>&1 || { tail $o/s128_${v}_$rep.log; exit 1; }
    echo "== $v $rep: $(tail -1 $o/s128_${v}_$rep.log)"
  done
done
