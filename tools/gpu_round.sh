#!/bin/bash
# Full GPU check on the box (run from the repo root via gpurun):
#   GPU parity tests -> default bench line -> rocprofv3 kernel stats -> PMC traffic.
# Every GPU step has its own time limit; the chain stops at the first failure.
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -m pytest tests -m gpu -q -rf -x > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err; rc=$?
echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd $R && bash tools/pmc_traffic.sh > $O/pmc.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -1 $O/pmc.log
exit $rc
