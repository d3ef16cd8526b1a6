# round 4: handle-ABI aggregate vs hardware queues (GPU_MAX_HW_QUEUES, launch slots follow it)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4l
mkdir -p $O
cd $R
for Q in 4 8 16 32; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/q$Q.json 2> $O/q$Q.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/q$Q.json'))['stream'];h=d['handles'];h={**h, **(h.get('batch') or {})};print('hwq=$Q one',d['one_handle']['value'],{k:h[k] for k in ('value','calls_per_launch','launch_us_avg','kernel_us_avg','slots_busy')})"
done
