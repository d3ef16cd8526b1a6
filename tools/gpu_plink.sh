#!/bin/bash
# parallel-prefix link: chunked parity tests (few-stream batches take it), one-stream probe
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pl}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_deflate64.py tests/test_zip.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/one_stream_probe.py > $O/one.log 2>&1; rc=$?
grep -v amdgpu.ids $O/one.log | tail -3
exit $rc
