#!/bin/bash
# lane-to-unit mapping experiment: parity with interleaving, C2 and C5 benches per mapping
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-lm}
mkdir -p $O
cd $R
ZS_LANE_MAP=1024 timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -1 $O/t.log
[ $rc -eq 0 ] || exit $rc
for m in 0 1024 768 256; do
  ZS_LANE_MAP=$m timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg > $O/c2_$m.json 2> $O/c2_$m.err || exit 1
  python3 -c "
import json;d=json.load(open('$O/c2_$m.json'));print('map $m c2',d['value'],d['ms_per_step'],d['roofline']['stages_ms_avg']['parse'])"
done
for m in 0 768; do
  ZS_LANE_MAP=$m timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg > $O/c5_$m.json 2> $O/c5_$m.err || exit 1
  python3 -c "
import json;d=json.load(open('$O/c5_$m.json'));print('map $m c5',d['value'],d['ms_per_step'],d['roofline']['stages_ms_avg']['parse'])"
done
