# round 4: stream leg (default worker life, then a long life) -- relaunch feedback check
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4y
mkdir -p $O
cd $R
show() { python3 -c "
import json;d=json.load(open('$1'))['stream'];print(d['one_handle']);print(d['handles'])"; }
timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/stream.json 2> $O/stream.err || exit $?
show $O/stream.json
ZS_PK_LIFE_MS=5000 timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/stream_life.json 2> $O/stream_life.err || exit $?
show $O/stream_life.json
