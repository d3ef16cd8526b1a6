#!/bin/bash
# chunked-path parity with the parse forced to each mode, then the one-stream probe
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pm}
mkdir -p $O
cd $R
ZS_PARSE=wave timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_deflate64.py tests/test_zip.py tests/test_gpu_stream.py -x -q --timeout 300 --timeout-method thread > $O/pytest_wave.log 2>&1; rc=$?
echo "wave-mode tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_wave.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/one_stream_probe.py > $O/one.log 2>&1; rc=$?
grep -v amdgpu.ids $O/one.log | tail -3
exit $rc
