#!/bin/bash
# expand kernel A/B: inflate parity tests on the default (expand2), then the short headline bench
# with expand2 and with the round-per-batch kernel (ZS_EXPAND=1)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-eab}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_pieces.py tests/test_zip.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in 2 1; do
  ZS_EXPAND=$v timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg > $O/bench_e$v.json 2> $O/bench_e$v.err; rc=$?
  echo "bench expand$v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json;d=json.load(open('$O/bench_e$v.json'))
print('value',d['value'],'ms',d['ms_per_step'],'ok',d['verified_bit_exact']);print(d['roofline']['stages_ms_avg'])"
done
