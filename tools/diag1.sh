#!/bin/bash
# dev: two-pass vs one-pass screen diagnostics (tools/scan_diag.py)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag1
NRK_LIB_PATH=news-recommendation-tc_amd/build_dev/libnrk.so timeout -k 10 200 python tools/scan_diag.py > gpurun_out/diag1/two.txt 2>&1
tail -4 gpurun_out/diag1/two.txt
timeout -k 10 200 python tools/scan_diag.py > gpurun_out/diag1/one.txt 2>&1
tail -4 gpurun_out/diag1/one.txt
NRK_LIB_PATH=news-recommendation-tc_amd/build_dev/libnrk.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/diag1/prof -o run -- python tools/scan_diag.py > /dev/null 2>&1
f=$(find gpurun_out/diag1/prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-220
