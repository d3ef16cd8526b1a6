# round 4: kernel split of the handle-ABI aggregate (one slot, gathered batches)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ZS_STREAM_SLOTS=1 ZS_STREAM_GATHER_US=200 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --only-stream --no-ref-perf > $O/stream.json 2> $O/stream.err; rc=$?
echo "rc=$rc"
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cat "$f" | cut -d, -f1-8 | head -20
