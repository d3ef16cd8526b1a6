#!/bin/bash
# round 4 check: deflate stream parity (level 0, output-full pull-on-demand,
# reference round-trip inputs), the inflate parity suite on the LXB parse,
# then the headline inflate leg A/B (default = ZS_LXB, variant lxb0) and the
# zlib-bytes deflate probe A/B (default = msearch work queue, variant msq0)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r4e}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread > $O/defl.log 2>&1; rc=$?
echo "deflate tests rc=$rc"; tail -3 $O/defl.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_pieces.py -x -q --timeout 300 --timeout-method thread > $O/infl.log 2>&1; rc2=$?
echo "inflate tests rc=$rc2"; tail -3 $O/infl.log
[ $rc2 -eq 0 ] || exit $rc2
for v in default lxb0 default lxb0; do
  L=""; [ "$v" = default ] || L=$R/zlib-streams_amd/libzstreams_mi355x_$v.so
  ZS_LIB=$L timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg --no-c5-leg > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/bench_$v.json'))
print('$v value',d['value'],'ms',d['ms_per_step'],'ok',d['verified_bit_exact'],d['roofline']['stages_ms_avg'])"
done
for v in default msq0 default msq0; do
  L=""; [ "$v" = default ] || L=$R/zlib-streams_amd/libzstreams_mi355x_$v.so
  ZS_LIB=$L timeout -k 10 300 python3 -u tools/zd_probe.py --streams 16 --mib 64 --level 6 --reps 2 > $O/probe_$v.log 2>&1 || exit $?
  echo "probe $v: $(tail -2 $O/probe_$v.log | tr '\n' ' ')"
done
exit $rc
