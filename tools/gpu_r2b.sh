#!/bin/bash
# Round-2 GPU check: parity tests, default bench line, C5 at 4096 streams,
# rocprofv3 kernel stats of the bench.  Each GPU step has its own limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r2b}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; head -c 600 $O/bench.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --workload c5 --c5-streams 4096 --steps 5 --no-cpu-baseline > $O/bench_c5_4096.json 2> $O/bench_c5.err; rc=$?
echo "c5 rc=$rc"; head -c 400 $O/bench_c5_4096.json; echo
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_rocprof.json 2> $O/bench_rocprof.err; rc=$?
echo "rocprof rc=$rc"
exit $rc
