#!/bin/bash
# deflate stream surface: probe (wall-clock) + rocprofv3 kernel stats of an L6 run
TAG=${1:-dsp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LEVELS=${LEVELS:-6} timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/dstream_probe.py ${MIB:-4} > $O/probe.log 2>&1; rc=$?
cat $O/probe.log
echo "rocprof rc=$rc"
head -30 $(find $O/prof -name '*kernel_stats.csv' | head -1)
exit $rc
