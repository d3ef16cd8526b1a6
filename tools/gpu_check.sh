#!/bin/bash
# coalesced checks: GPU suite, then C5 (4096 mixed raw/gzip) and the compress leg stage split
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ck}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_all.log 2>&1; rc=$?
echo "gpu suite rc=$rc"; tail -3 $O/gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c5 --steps 3 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg > $O/c5.json 2> $O/c5.err; rc=$?
echo "c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.load(open('$O/c5.json'))
print('c5 value',d['value'],'ms',d['ms_per_step'],'ok',d['verified_bit_exact'],d['path_stats']);print(d['roofline']['stages_ms_avg'])"
timeout -k 10 400 python -u bench.py --steps 3 --no-cpu-baseline --no-deflate64 --no-stream-leg > $O/c2.json 2> $O/c2.err; rc=$?
echo "c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json;d=json.load(open('$O/c2.json'))
print('c2 value',d['value'],'ms',d['ms_per_step'],'ok',d['verified_bit_exact']);print(d['roofline']['stages_ms_avg']);c=d['compress'];print('compress',c['value'],c.get('stages_ms_avg') or c.get('roofline',{}).get('stages_ms_avg'))"
