# round 4: the new stream test alone
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4t2
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -k "more_handles or relaunch" -v --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
echo rc=$rc; grep -E "PASS|FAIL|Error|assert" $O/t.log | head -20
