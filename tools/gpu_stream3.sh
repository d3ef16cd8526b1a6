#!/bin/bash
# handle-ABI stream path: stream parity tests (Appendix C traces, JS schedules,
# zlib-ABI calls, concurrent handles), then the bench's stream leg alone.
TAG=${1:-st}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_pieces.py -x -v -rf --timeout 200 --timeout-method thread > $O/pytest_stream.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_stream.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --only-stream > $O/stream.json 2> $O/stream.err; rc=$?
echo "stream rc=$rc"; cat $O/stream.json
exit $rc
