#!/bin/bash
# deflate parity on the box: the GPU deflate tests (zlib bytes, stream calls vs host zlib), then the smoke
TAG=${1:-dz}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py -v -rf --timeout 300 --timeout-method thread > $O/pytest_deflate.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_deflate.log | tail -40
exit $rc
