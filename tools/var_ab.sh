#!/bin/bash
# A/B bench of library variants (C2 inflate leg only): tools/var_ab.sh OUT v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-var}; shift
mkdir -p $O
cd $R
for v in "$@"; do
  L=""; [ "$v" = default ] || L=$R/zlib-streams_amd/libzstreams_mi355x_$v.so
  ZS_LIB=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ref-perf --no-compress --no-deflate64 --no-stream-leg --no-c5-leg > $O/bench_$v.json 2> $O/bench_$v.err; rc=$?
  echo "bench $v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json;d=json.load(open('$O/bench_$v.json'))
print('value',d['value'],'ms',d['ms_per_step'],'ok',d['verified_bit_exact']);print(d['roofline']['stages_ms_avg'])"
done
