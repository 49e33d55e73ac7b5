#!/bin/bash
# Round evidence in one GPU-box call (dev tool): GPU parity tests, the default
# bench, its rocprofv3 kernel-trace summary, and the FETCH_SIZE / WRITE_SIZE
# passes behind roofline.traffic.  usage: tools/round_profile.sh TAG
set -o pipefail
TAG=${1:-rp}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_prof.log 2>&1 || { tail -30 $O/bench_prof.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c -d $O/rec_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-din --no-cpu-baseline > $O/rec_$c.log 2>&1 || { tail -5 $O/rec_$c.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc $c -d $O/din_$c -o run --output-format csv -- python3 tools/din_prof.py 2 > $O/din_$c.log 2>&1 || { tail -5 $O/din_$c.log; exit 1; }
done
echo done
