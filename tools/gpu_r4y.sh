# round 4: stream windows (J3 walks, 8 consecutive offsets per thread) + tree build without scratch arrays
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4y
mkdir -p $O
cd $R
bash tools/gpu_r4x.sh || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread > $O/deflate_tests.log 2>&1; rc=$?
echo "deflate tests rc=$rc"; tail -2 $O/deflate_tests.log
[ $rc -eq 0 ] || exit $rc
for K in random lines; do
  LEVELS=6 KINDS=$K timeout -k 10 200 python3 -u tools/dstream_probe.py 4 2>&1 | grep GPU || exit 1
done
timeout -k 10 300 python3 tools/zd_probe.py 2>&1 | grep "zlib-bytes"
