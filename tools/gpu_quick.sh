# GPU parity tests, then a short bench (inflate leg only) and the parse/expand counters
mkdir -p gpurun_out/q
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/q/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -6 gpurun_out/q/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-compress --no-deflate64 > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/q/bench.json'));print(d['value'],d['ms_per_step'],d['verified_bit_exact'],d['roofline']['stages_ms_avg'],d['path_stats'])"
[ $rc -eq 0 ] || exit $rc
ZS_LIB=$PWD/zlib-streams_amd/libzstreams_mi355x_prof.so timeout -k 10 300 python -u tools/kprof_run.py --out gpurun_out/q/kprof.json > gpurun_out/q/kprof.log 2>&1; rc=$?
echo "kprof rc=$rc"; python3 -c "import json;d=json.load(open('gpurun_out/q/kprof.json'))['derived'];print({k:d[k] for k in ('ok','parse_cycles_per_wave','parse_cycles_max','parse_cycles_per_wave_step','parse_lane_util','expand_cycles_per_round')})"
