#!/bin/bash
# dev: 8-shard config-4 replay + its kernel stats
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; mkdir -p $o
timeout -k 10 400 python3 tools/catalog_replay.py 8 > $o/replay.log 2>&1 || { tail -20 $o/replay.log; exit 1; }
tail -12 $o/replay.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o/p -o run -- python3 tools/catalog_replay.py 8 > $o/replay_prof.log 2>&1 || exit 1
python3 tools/kstats.py $o/p/run_kernel_stats.csv 12
