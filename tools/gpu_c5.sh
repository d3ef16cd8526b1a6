# GPU parity tests, then the C5 (many mixed 4 MiB streams) bench
mkdir -p gpurun_out/c5
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/c5/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/c5/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c5 --c5-streams 1024 --steps 3 --cpu-seconds 3 > gpurun_out/c5/bench.json 2> gpurun_out/c5/bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/c5/bench.json
