#!/bin/bash
# handle-ABI aggregate A/B: the bench stream leg (one handle, 64 handles on
# native threads) under ZS_STREAM_SLOTS = 1 / 2 / 4 launch slots
TAG=${1:-slots}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for SG in ${CASES:-4:0 2:0 1:0 1:30 2:30 4:30}; do
  S=${SG%:*}; G=${SG#*:}
  ZS_STREAM_SLOTS=$S ZS_STREAM_GATHER_US=$G timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/stream_s${S}_g$G.json 2> $O/stream_s${S}_g$G.err || exit $?
  echo "slots=$S gather=$G $(python3 -c "import json;d=json.load(open('$O/stream_s${S}_g$G.json'))['stream'];print('one',d['one_handle']['value'],'agg',d['handles']['value'],'cpl',(d['handles'].get('batch') or {}).get('calls_per_launch'))")"
done
