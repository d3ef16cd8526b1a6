#!/bin/bash
# deflate stream surface: the deflate GPU tests, then the stream probe (L6 and L1)
TAG=${1:-ds}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -q -rf -x --timeout 600 --timeout-method thread > $O/pytest_deflate.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_deflate.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/dstream_probe.py ${MIB:-16} > $O/probe.log 2>&1; rc=$?
cat $O/probe.log
exit $rc
