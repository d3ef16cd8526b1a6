#!/bin/bash
# deflate parity tests + bench compress legs (zlib bytes and fast)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2c
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_deflate64.py -x -v --timeout 300 --timeout-method thread > $O/pytest_deflate.log 2>&1; rc=$?
echo "deflate tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" $O/pytest_deflate.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 3 --no-cpu-baseline --no-deflate64 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -3 $O/bench.err
python3 -c "
import json;d=json.load(open('$O/bench.json'));c=d['compress'];f=c['fast_mode']
print('inflate',d['value'])
for x in (c,f): print(x['mode'],x['value'],x['ratio'],x['bytes_identical_to_zlib'],x['roundtrip_verified'],x['roofline']['stages_ms_avg'])"
exit $rc
