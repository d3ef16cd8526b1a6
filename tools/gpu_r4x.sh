# round 4: stream windows keep J3 (shorter per-thread chain walks) -- inflate + stream tests, stream leg
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4x
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_inflate.py tests/test_gpu_pieces.py tests/test_gpu_deflate64.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/stream.json 2> $O/stream.err || exit $?
python3 -c "
import json;d=json.load(open('$O/stream.json'))['stream'];h=d['handles'];print('one',d['one_handle']);print({k:h[k] for k in h if k!='stream'})"
