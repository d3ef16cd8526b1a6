#!/bin/bash
# round 4 final: GPU suite -> PMC traffic -> driver-shaped bench (reading that traffic) -> rocprofv3 kernel stats,
# all on the library in the tree (each GPU step under its own limit; stops at the first failure)
TAG=${1:-r4final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
PMC_TAG=$TAG bash tools/pmc_traffic.sh && [ -s $R/gpurun_out/pmc/pmc_traffic.json ] || exit 1
cd $R
t0=$SECONDS
timeout -k 10 500 python3 bench.py --traffic-json $R/gpurun_out/pmc/pmc_traffic.json > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc wall_s=$((SECONDS - t0))"
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);s=d['stream'];print(d['value'], d['roofline']['traffic'], d['roofline'].get('traffic_source',{}).get('same_library_build'), 'C3', d['compress']['value'], 'one', s['one_handle']['value'], 'agg', s['handles']['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ref-perf > $O/bench_rocprof.json 2> $O/bench_rocprof.err; rc=$?
echo "rocprof rc=$rc"
find $O/prof -name "*kernel_trace.csv" -delete
[ $rc -eq 0 ] || exit $rc

