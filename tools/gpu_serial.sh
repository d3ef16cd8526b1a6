# serial-decoder change check: GPU parity tests, then the timing probe
mkdir -p gpurun_out/ser
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ser/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -15 gpurun_out/ser/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/serial_probe.py > gpurun_out/ser/probe.log 2>&1; rc=$?
echo "probe rc=$rc"; cat gpurun_out/ser/probe.log

ZS_LIB=$PWD/zlib-streams_amd/libzstreams_mi355x_prof.so timeout -k 10 120 python -u tools/serial_kprof.py > gpurun_out/ser/kprof.log 2>&1; rc=$?
echo "kprof rc=$rc"; cat gpurun_out/ser/kprof.log
