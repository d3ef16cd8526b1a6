#!/bin/bash
# deflate_fast (levels 1..3) on the box: stage probe at each level (bytes vs host
# zlib), then the deflate GPU tests that cover levels 1..3.  Each GPU step has its
# own time limit; the chain stops at the first failure.
TAG=${1:-fl}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for lv in 1 2 3; do
  timeout -k 10 180 python3 -u tools/zd_probe.py --streams 2 --mib 16 --level $lv --reps 1 >> $O/probe.log 2>&1 || { echo "probe L$lv failed"; tail -5 $O/probe.log; exit 1; }
done
cat $O/probe.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -v -rf -x --timeout 600 --timeout-method thread > $O/pytest_deflate.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_deflate.log | tail -45
exit $rc
