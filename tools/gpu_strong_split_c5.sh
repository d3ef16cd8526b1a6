#!/bin/bash
# configs[4] scaling prediction on ONE GPU: the strong-split share of the fixed
# 4096 x 4 MiB batch that rank 0 (and the last rank) decodes at 1/2/4/8 ranks
# (LPT, shard.bench_shard), inflate only, with its parse / link modes.
TAG=${1:-split_c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for W in 1 2 4 8; do
  for RK in 0 $((W - 1)); do
    [ $W -eq 1 ] && [ $RK -ne 0 ] && continue
    timeout -k 10 300 python3 -u bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline --no-stream-leg --sim-world $W --sim-rank $RK \
      > $O/c5_w${W}_r${RK}.json 2> $O/c5_w${W}_r${RK}.err || exit $?
    echo "W=$W rank=$RK $(python3 -c "import json;d=json.load(open('$O/c5_w${W}_r${RK}.json'));print(d['ms_per_step'], d['config']['streams_rank0'], d['verified_bit_exact'], d['path_stats']['parse'], d['path_stats']['link'])")"
  done
done
