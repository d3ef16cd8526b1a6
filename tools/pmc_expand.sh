#!/bin/bash
# SQ counters of the expand kernel on the headline workload: two rocprofv3 --pmc passes, kernel trace only
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pf}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg"
K="--kernel-include-regex ${KREGEX:-zs_expand}"
timeout -k 10 300 rocprofv3 --kernel-trace $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p1 -- python3 $B > $OUT/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace $K --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $OUT/p2 -o p2 -- python3 $B > $OUT/p2.log 2>&1
rc=$?
echo "pmc rc=$rc"
python3 $R/tools/pmc_sq_summary.py $OUT
exit $rc
