# round 4: stream kernel batched slowdown -- pinned-array views vs device copies
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4j
mkdir -p $O
cd $R
for V in 1 0; do
  ZS_STREAM_VIEWS=$V ZS_STREAM_SLOTS=1 ZS_STREAM_GATHER_US=200 timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/v$V.json 2> $O/v$V.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/v$V.json'))['stream'];h=d['handles'];h={**h, **(h.get('batch') or {})};print('views=$V one',d['one_handle']['value'],{k:h[k] for k in ('value','calls_per_launch','launch_us_avg','kernel_us_avg','gather_us_avg','slots_busy')})"
done
