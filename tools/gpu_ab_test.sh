#!/bin/bash
# inflate parity (split + deflate64 block-parallel tests) on the default build, then the
# C2 A/B bench of the named variants: tools/gpu_ab_test.sh OUT v1 v2 ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ab}; shift
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_deflate64.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -6
[ $rc -eq 0 ] || exit $rc
bash tools/var_ab.sh "$(basename $O)" "$@"
