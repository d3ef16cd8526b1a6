#!/bin/bash
# A/B of library variants on the handle-ABI stream leg only: tools/stream_ab.sh OUT v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-sab}; shift
mkdir -p $O
cd $R
for v in "$@"; do
  L=""; [ "$v" = default ] || L=$R/zlib-streams_amd/libzstreams_mi355x_$v.so
  ZS_LIB=$L timeout -k 10 400 python -u bench.py --only-stream --no-cpu-baseline > $O/s_$v.json 2> $O/s_$v.err; rc=$?
  echo "stream $v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json;d=json.load(open('$O/s_$v.json'));s=d.get('stream',d)
print('$v', s['one_handle']['value'], s['handles']['value'], s['reference_perf_workload']['gpu']['decompress_only'])"
done
