# round 4: handle-ABI aggregate timing (slots x gather), stream leg only
mkdir -p gpurun_out/r4h
CASES="4:0 1:0 1:200 1:1000 4:200 2:200" bash tools/gpu_stream_slots.sh r4h/slots || exit $?
for f in gpurun_out/r4h/slots/*.json; do python3 -c "
import json;d=json.load(open('$f'))['stream']['handles'];d={**d, **(d.get('batch') or {})};print('$f'.split('/')[-1], {k:d[k] for k in ('value','calls_per_launch','launch_us_avg','kernel_us_avg','gather_us_avg','slots_busy')})"; done
