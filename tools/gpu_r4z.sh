# round 4: stream leg twice with the driver's per-thread split
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4z
mkdir -p $O
cd $R
for k in 1 2; do
ZS_JS_DRIVE_PROF=1 timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/stream$k.json 2> $O/stream$k.err || exit $?
python3 -c "
import json;d=json.load(open('$O/stream$k.json'))['stream'];h=d['handles'];print('one',d['one_handle']['value'],{k:h[k] for k in h if k.startswith('persistent') or k=='value'})"
grep js_drive $O/stream$k.err
done
