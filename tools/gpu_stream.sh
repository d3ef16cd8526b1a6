mkdir -p gpurun_out/st1
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 120 --timeout-method thread > gpurun_out/st1/pytest_stream.log 2>&1; rc=$?
echo "stream rc=$rc"; tail -30 gpurun_out/st1/pytest_stream.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/st1/pytest_gpu.log 2>&1; rc=$?
echo "gpu rc=$rc"; tail -5 gpurun_out/st1/pytest_gpu.log
