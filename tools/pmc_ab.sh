#!/bin/bash
# HBM traffic (tools/pmc_traffic.sh) of library variants: tools/pmc_ab.sh OUT v1 v2 ... (default = the in-tree build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmcab}; shift
mkdir -p $O
cd $R
for v in "$@"; do
  L=""; [ "$v" = default ] || L=$R/zlib-streams_amd/libzstreams_mi355x_$v.so
  ZS_LIB=$L PMC_OUT=$O/$v PMC_TAG=ab_$v bash tools/pmc_traffic.sh > $O/$v.log 2>&1; rc=$?
  echo "pmc $v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json;d=json.load(open('$O/$v/pmc_traffic.json'));k=d.get('per_kernel',d.get('kernels'))
print('$v', d['hbm_bytes_per_launch'], {n:(v['read_bytes'],v['write_bytes']) for n,v in k.items() if n in ('zs_split_kernel','zs_walk_kernel')})"
done
