#!/bin/bash
# GPU suite on the box: pytest -m gpu, smoke(), a short bench.  Usage: tools/gpu_suite.sh OUTDIR [pytest args]
out=gpurun_out/$1; shift
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 150 --timeout-method thread "$@" > "$out/pytest.log" 2>&1
rc=$?
tail -15 "$out/pytest.log"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > "$out/bench.json" 2> "$out/bench.err"
rc2=$?
tail -3 "$out/bench.err"; cat "$out/bench.json"
exit $(( rc > rc2 ? rc : rc2 ))
