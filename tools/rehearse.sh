#!/bin/bash
# One-GPU rehearsal of bench.py's N-rank layouts (config-4 catalog-sharded
# recall, DIN batches round-robin): N ranks share cuda:0 over gloo (host-
# staged collectives).  Correctness of the launch / layout / exchange path,
# not a measurement.  usage: tools/rehearse.sh TAG "2 3"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-reh}; mkdir -p $O
for n in ${2:-2 3}; do
  timeout -k 10 600 python -u bench.py --gpus $n --backend gloo --steps 2 --warmup 1 --no-cpu-baseline --no-plugins \
    --no-itemcf --din-steps 2 --din-warmup 1 > $O/bench_$n.log 2>&1 || { tail -30 $O/bench_$n.log; exit 1; }
  grep -v "^E2026\|^W2026" $O/bench_$n.log | tail -3 | cut -c1-900
done
