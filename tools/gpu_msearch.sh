#!/bin/bash
# zlib-bytes deflate search A/B on the box: the deflate GPU tests with the
# demand-driven search (zs_zd_msearch_kernel, default), then the L6 stage probe
# (16 x 64 MiB, bytes checked against host zlib) with it and with
# ZS_ZD_MATCH=all (zs_zd_match_kernel: every position, both budgets).
TAG=${1:-ms}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py -x -v -rf --timeout 300 --timeout-method thread > $O/pytest_deflate.log 2>&1; rc=$?
echo "deflate tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_deflate.log | tail -6
[ $rc -eq 0 ] || exit $rc
for lv in ${LEVELS:-6}; do
  for m in demand all; do
    E=""; [ $m = all ] && E=all
    ZS_ZD_MATCH=$E timeout -k 10 300 python3 -u tools/zd_probe.py --streams 16 --mib 64 --level $lv --reps 2 > $O/probe_L${lv}_$m.log 2>&1; rc=$?
    echo "probe L$lv $m rc=$rc"; tail -2 $O/probe_L${lv}_$m.log
    [ $rc -eq 0 ] || exit $rc
  done
done
