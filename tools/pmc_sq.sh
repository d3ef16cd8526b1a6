#!/bin/bash
# SQ instruction / wait counters for the lane (parse) and expand kernels on the
# bench workload: three rocprofv3 --pmc passes, kernel trace only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-sq}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-compress --no-deflate64 --no-stream-leg --no-c5-leg --no-ref-perf"
K="--kernel-include-regex ${K_RE:-zs_lane_kernel|zs_expand_kernel|zs_find_kernel|zs_link_kernel|zs_emit_kernel}"
timeout -k 10 400 rocprofv3 --kernel-trace $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES --output-format csv -d $OUT/p1 -o p1 -- python3 $B > $OUT/p1.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace $K --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $OUT/p2 -o p2 -- python3 $B > $OUT/p2.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace $K --pmc SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_LDS_ADDR_CONFLICT --output-format csv -d $OUT/p3 -o p3 -- python3 $B > $OUT/p3.log 2>&1
echo "pmc rc=$?"
