# round 4: deflate_slow merges at any no-pending-match state -- deflate tests, then the stream-surface timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4t
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread > $O/deflate_tests.log 2>&1; rc=$?
echo "deflate tests rc=$rc"; tail -3 $O/deflate_tests.log
[ $rc -eq 0 ] || exit $rc
for K in random lines zipf; do
  LEVELS=6 KINDS=$K timeout -k 10 200 python3 -u tools/dstream_probe.py 4 2>&1 | grep GPU || exit 1
done
timeout -k 10 300 python3 tools/zd_probe.py > $O/zd_probe.log 2>&1; echo "zd_probe rc=$?"; tail -5 $O/zd_probe.log
