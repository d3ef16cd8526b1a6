#!/bin/bash
# stream kernel profile: in-kernel counters (profiling build), then rocprofv3 kernel stats of the product build
TAG=${1:-sp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_prof.so timeout -k 10 200 python3 tools/stream_probe.py 16 > $O/probe_prof.log 2>&1; rc=$?
cat $O/probe_prof.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/stream_probe.py 16 > $O/probe_rocprof.log 2>&1; rc=$?
cat $O/probe_rocprof.log | tail -3
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -8 "$f"
exit $rc
