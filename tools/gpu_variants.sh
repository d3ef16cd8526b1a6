#!/bin/bash
# A/B of library variants: inflate parity tests on the default build, then the short
# headline bench (inflate leg) on the default build and on each named variant
# (zlib-streams_amd/libzstreams_mi355x_NAME.so, tools/build_variant.sh)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-var}; shift
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_pieces.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -6
[ $rc -eq 0 ] || exit $rc
for v in default "$@"; do
  L=""; [ "$v" = default ] || L=$R/zlib-streams_amd/libzstreams_mi355x_$v.so
  ZS_LIB=$L timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg > $O/bench_$v.json 2> $O/bench_$v.err; rc=$?
  echo "bench $v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json;d=json.load(open('$O/bench_$v.json'))
print('value',d['value'],'ms',d['ms_per_step'],'ok',d['verified_bit_exact']);print(d['roofline']['stages_ms_avg'])"
done
