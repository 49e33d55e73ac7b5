#!/bin/bash
# round-6 dev: SQ counters of the dim-128 refine (tools/scan128.py, 100k users)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
o=gpurun_out/r6p; mkdir -p $o
set -o pipefail
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $o/pmc -o run --output-format csv -- python3 tools/scan128.py 100000 > $o/pmc.log 2>&1 || { tail $o/pmc.log; exit 1; }
