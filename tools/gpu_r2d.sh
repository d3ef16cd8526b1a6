#!/bin/bash
# Round-2 re-entry check: smoke, full GPU parity suite, default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2d
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; head -c 800 $O/bench.json; echo
exit $rc
