# round 4: persistent worker timing (stream leg only)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4n
mkdir -p $O
cd $R
ZS_JS_DRIVE_PROF=1 timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/stream.json 2> $O/stream.err || exit $?
python3 -c "
import json;d=json.load(open('$O/stream.json'))['stream'];h=d['handles'];print('one',d['one_handle']);print({k:h[k] for k in h if k!='stream'})"
grep js_drive $O/stream.err
