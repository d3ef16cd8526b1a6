#!/bin/bash
# Checkpoint run on the GPU box (from the repo root via gpurun):
#   all GPU parity tests -> default bench line -> rocprofv3 kernel stats of the bench -> C5 line.
# Every GPU step has its own time limit; the chain stops at the first failure.
TAG=${1:-ckpt}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err; rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 400 python3 -u bench.py --workload c5 --steps 3 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg > $O/c5.json 2> $O/c5.err; rc=$?
echo "c5 rc=$rc"; cat $O/c5.json
exit $rc
