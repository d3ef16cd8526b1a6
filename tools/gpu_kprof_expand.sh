#!/bin/bash
# expand2 phase counters on the headline workload (profiling build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-kpe}
mkdir -p $O
cd $R
ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_prof.so timeout -k 10 300 python -u tools/kprof_run.py --out $O/kprof.json > $O/kprof.log 2>&1; rc=$?
echo "kprof rc=$rc"
python3 -c "
import json;d=json.load(open('$O/kprof.json'))
r=d['raw'];print({k:r[k] for k in r if k.startswith('e_')})
print({k:v for k,v in d['derived'].items() if k.startswith('expand') or k=='ok'})"
exit $rc
