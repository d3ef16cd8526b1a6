#!/bin/bash
# A/B bench (C2 inflate leg) of environment settings: tools/env_ab.sh OUT "" "ZS_X=1" "ZS_X=2 ZS_Y=0" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-envab}; shift
mkdir -p $O
cd $R
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ref-perf --no-compress --no-deflate64 --no-stream-leg --no-c5-leg > $O/bench_$i.json 2> $O/bench_$i.err; rc=$?
  echo "bench [$e] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json;d=json.load(open('$O/bench_$i.json'))
print('value',d['value'],'ms',d['ms_per_step'],'ok',d['verified_bit_exact']);print(d['roofline']['stages_ms_avg'])"
done
