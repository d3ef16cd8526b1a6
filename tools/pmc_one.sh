#!/bin/bash
# one rocprofv3 SQ counter pass over the bench for kernels matching $2
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-one}; KRE=${2:-zs_find_kernel}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --kernel-include-regex "$KRE" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p1 -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/p1.log 2>&1
echo "pmc rc=$?"
