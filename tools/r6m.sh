#!/bin/bash
# round-6 dev: pipelined recall steps (next tower beside select + finish) vs serial
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6m; mkdir -p $o
set -o pipefail
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-din --no-itemcf --no-plugins > $o/bench_$rep.json 2> $o/bench_$rep.err || { tail $o/bench_$rep.err; exit 1; }
  echo "== $rep: $(grep -o '"ms_per_step": [0-9.]*\|"ms_per_step_serial": [0-9.]*\|"phase_ms": {[^}]*}' $o/bench_$rep.json | tr '\n' ' ')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-din --no-itemcf --no-plugins > $o/prof.log 2>&1 || { tail $o/prof.log; exit 1; }
