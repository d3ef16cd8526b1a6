# round 4: persistent stream worker -- stream tests, then the stream leg
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4m
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_inflate.py -k "not chunked and not c2_ and not c5_ and not segmented and not large and not gzip_zlib_checks" -x -v --timeout 120 --timeout-method thread > $O/stream_tests.log 2>&1; rc=$?
echo "stream tests rc=$rc"; grep -E "passed|failed|FAIL|Error" $O/stream_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/stream.json 2> $O/stream.err || exit $?
python3 -c "
import json;d=json.load(open('$O/stream.json'))['stream'];h=d['handles'];print('one',d['one_handle'],{k:h[k] for k in h if k!='stream'})"
