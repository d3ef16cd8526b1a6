#!/bin/bash
# Scaling prediction on ONE GPU: rank 0's strong-split share of the 64 x 64 MiB
# batch at 1/2/4/8 ranks (LPT by compressed size), inflate leg only, plus the
# parse mode / link mode each share takes.  Each run has its own time limit.
TAG=${1:-split}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for W in 1 2 4 8; do
  timeout -k 10 240 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-compress --no-deflate64 \
    --no-stream-leg --sim-world $W > $O/split_$W.json 2> $O/split_$W.err || exit $?
  echo "W=$W $(python3 -c "import json;d=json.load(open('$O/split_$W.json'));print(d['ms_per_step'], d['config']['streams_rank0'], d['path_stats'])")"
done
