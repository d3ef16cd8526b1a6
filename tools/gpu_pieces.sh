#!/bin/bash
# long streams in pieces: the piece tests, then the whole GPU suite
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pc}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_pieces.py -x -v --timeout 300 --timeout-method thread > $O/pieces.log 2>&1; rc=$?
echo "piece tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/pieces.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_all.log 2>&1; rc=$?
echo "gpu suite rc=$rc"; tail -3 $O/gpu_all.log
exit $rc
