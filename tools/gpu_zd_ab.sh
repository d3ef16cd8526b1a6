#!/bin/bash
# A/B of zlib-bytes deflate library variants (tools/build_variant.sh with
# SRC=deflate_zlib): the deflate GPU tests on each variant, then the L6 stage
# probe (16 x 64 MiB, bytes checked against host zlib) on the default build
# and each variant.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-zdab}; shift
mkdir -p $O
cd $R
for v in "$@"; do
  ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 300 --timeout-method thread -k "not calls_are_zlibs or 6" > $O/pytest_$v.log 2>&1; rc=$?
  echo "tests $v rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_$v.log | tail -4
  [ $rc -eq 0 ] || exit $rc
done
for v in default "$@"; do
  L=""; [ "$v" = default ] || L=$R/zlib-streams_amd/libzstreams_mi355x_$v.so
  ZS_LIB=$L timeout -k 10 300 python3 -u tools/zd_probe.py --streams 16 --mib 64 --level ${LEVEL:-6} --reps 2 > $O/probe_$v.log 2>&1; rc=$?
  echo "probe $v rc=$rc"; tail -1 $O/probe_$v.log
  [ $rc -eq 0 ] || exit $rc
done
