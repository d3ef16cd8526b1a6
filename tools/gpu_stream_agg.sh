#!/bin/bash
# aggregate handle-ABI leg alone: 1 handle, then 64 handles at 1/2/4 launch
# slots; then the 64-handle default under rocprofv3 kernel trace
TAG=${1:-sa}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 100 python3 tools/stream_agg_probe.py 1 16 > $O/agg_1.log 2>&1 && cat $O/agg_1.log || exit 1
for s in 1 2 4; do
  ZS_STREAM_SLOTS=$s timeout -k 10 100 python3 tools/stream_agg_probe.py 64 4 > $O/agg_64_s$s.log 2>&1 || exit 1
  echo "slots=$s"; cat $O/agg_64_s$s.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/stream_agg_probe.py 64 4 > $O/agg_rocprof.log 2>&1; rc=$?
tail -2 $O/agg_rocprof.log
exit $rc
