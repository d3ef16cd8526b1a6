#!/bin/bash
# stream-surface check: GPU stream parity tests + the handle-ABI stream leg
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-s1}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --only-stream > $O/stream.json 2> $O/stream.err; rc=$?
echo "stream rc=$rc"; cat $O/stream.json
exit $rc
