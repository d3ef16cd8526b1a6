mkdir -p gpurun_out/r4g
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py -v --timeout 300 --timeout-method thread -k "level0 or roundtrip_inputs or small_out_buffer or output_full or tiny_calls or stream_calls or flush_loops" > gpurun_out/r4g/defl.log 2>&1
rc=$?; echo deflate rc=$rc; grep -E "PASS|FAIL" gpurun_out/r4g/defl.log | tail -40
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_stream_slots.sh r4g/slots || exit $?
bash tools/gpu_strong_split_c5.sh r4g/split_c5
