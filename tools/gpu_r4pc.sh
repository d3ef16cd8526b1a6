# round 4: parse walks through a per-thread LDS window of the match tables -- deflate tests, stream surface, batch
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4pc
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread > $O/deflate_tests.log 2>&1; rc=$?
echo "deflate tests rc=$rc"; tail -2 $O/deflate_tests.log
[ $rc -eq 0 ] || exit $rc
for K in random lines zipf; do
  LEVELS=6 KINDS=$K timeout -k 10 200 python3 -u tools/dstream_probe.py 4 2>&1 | grep GPU || exit 1
done
timeout -k 10 300 python3 tools/zd_probe.py 2>&1 | grep "zlib-bytes"
