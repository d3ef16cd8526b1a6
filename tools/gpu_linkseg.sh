#!/bin/bash
# segmented link (zs_linkseg_kernel): the inflate / pieces / ZIP GPU tests
# (batches of 5..64 streams take it), then the headline bench with it and with
# ZS_LINKSEG=0 (the per-stream serial link) for the stage split
TAG=${1:-ls}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_pieces.py tests/test_zip.py tests/test_gpu_stream.py -x -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in seg serial; do
  env $( [ $v = serial ] && echo ZS_LINKSEG=0 ) timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg > $O/bench_$v.json 2> $O/bench_$v.err; rc=$?
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json;d=json.load(open('$O/bench_$v.json'));print('$v',d['value'],d['ms_per_step'],d['verified_bit_exact'],d['path_stats']['link'],d['roofline']['stages_ms_avg'])"
done
