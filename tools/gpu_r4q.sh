# round 4: rocprofv3 kernel stats of the bench (headline + legs, no reference perf workload),
# then the PMC traffic passes on the same library
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ref-perf > $O/bench_rocprof.json 2> $O/bench_rocprof.err; rc=$?
echo "rocprof rc=$rc"
find $O/prof -name "*kernel_trace.csv" -delete
[ $rc -eq 0 ] || exit $rc
cd $R
PMC_TAG=r4q bash tools/pmc_traffic.sh
cat gpurun_out/pmc/pmc_traffic.json | head -40
