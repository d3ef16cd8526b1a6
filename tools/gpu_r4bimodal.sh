# round 4: 64-handle stream leg three times with the driver's per-thread breakdown (ZS_JS_DRIVE_PROF)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4bi
mkdir -p $O
cd $R
for i in ${RUNS:-1 2 3}; do
  ZS_JS_DRIVE_PROF=${ZS_JS_DRIVE_PROF:-1} timeout -k 10 300 python3 -u bench.py --only-stream --no-ref-perf > $O/s$i.json 2> $O/s$i.err || exit $?
  python3 -c "
import json;h=json.load(open('$O/s$i.json'))['stream']['handles'];print($i,h['value'],h['persistent_launches'],h['persistent_wait_us_avg'])"
  grep -A70 "js_drive" $O/s$i.err | tail -66
done
