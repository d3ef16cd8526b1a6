#!/bin/bash
# Full GPU check on the box (run from the repo root via gpurun):
#   GPU parity tests -> driver-shaped bench line (--steps 20 --warmup 5, wall time
#   recorded) -> rocprofv3 kernel stats.  Every GPU step has its own time limit;
#   the chain stops at the first failure.  PMC traffic: tools/pmc_traffic.sh.
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
t0=$SECONDS
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
t1=$SECONDS
echo "bench rc=$rc wall_s=$((t1 - t0))" | tee $O/bench_wall.txt; cat $O/bench.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err; rc=$?
echo "rocprof rc=$rc"
exit $rc
