#!/bin/bash
# dev: kernel stats of a config-5 fused step (250k users x 5M items)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/p -o run -- python3 bench.py --fused --fused-users 250000 --no-cpu-baseline --steps 1 --warmup 1 > $o/fused.log 2>&1 || { tail -20 $o/fused.log; exit 1; }
tail -1 $o/fused.log | grep -o '"phase_ms": {[^}]*}'
python3 tools/kstats.py $o/p/run_kernel_stats.csv 14
