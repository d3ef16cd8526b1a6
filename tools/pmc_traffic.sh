#!/bin/bash
# HBM traffic of the inflate pipeline on the bench workload: two rocprofv3 PMC
# passes (FETCH_SIZE, WRITE_SIZE), kernel trace only (no sys/runtime traces).
# Run on the GPU box from the repo root; writes $PMC_OUT (default gpurun_out/pmc)/pmc_traffic.json
# (copy it into profiles/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${PMC_OUT:-$R/gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg --no-c5-leg"
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $B > $OUT/fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $B > $OUT/write.log 2>&1 && \
python3 $R/tools/pmc_traffic.py $(find $OUT/fetch -name "*counter_collection.csv" | head -1) \
  $(find $OUT/write -name "*counter_collection.csv" | head -1) $OUT/pmc_traffic.json ${PMC_TAG:-}
echo "pmc rc=$?"
