#!/bin/bash
# inflate-pipeline iteration: chunked-path parity tests + short headline bench (stage split)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-iq}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_deflate64.py tests/test_zip.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"
python3 -c "
import json;d=json.load(open('$O/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'ok',d['verified_bit_exact'],d['path_stats']);print(d['roofline']['stages_ms_avg'])"
exit $rc
