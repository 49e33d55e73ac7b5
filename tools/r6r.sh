#!/bin/bash
# round-6 dev: SQ counters of the ItemCF recall kernels (bench ItemCF leg)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6r; mkdir -p $o
set -o pipefail
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $o/pmc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-din --no-plugins > $o/pmc.log 2>&1 || { tail $o/pmc.log; exit 1; }
