# round 4: persistent worker + deferred state init -- stream tests, deflate round trips, stream leg
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4o
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_inflate.py tests/test_gpu_deflate.py -k "stream or zlib_abi or roundtrip_inputs or appendix or js_schedule or concurrent or handle" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAIL|Error" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
ZS_JS_DRIVE_PROF=1 timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/stream.json 2> $O/stream.err || exit $?
python3 -c "
import json;d=json.load(open('$O/stream.json'))['stream'];h=d['handles'];print('one',d['one_handle']);print({k:h[k] for k in h if k!='stream'})"
grep js_drive $O/stream.err
