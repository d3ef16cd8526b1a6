#!/bin/bash
# usage: run_gpu.sh TAG [bench args...]
TAG=$1; shift
/usr/local/graft/bin/gpurun --timeout 900 -- "mkdir -p gpurun_out; timeout -k 10 400 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_$TAG.log 2>&1; rc=\$?; echo pytest rc=\$rc; if [ \$rc -le 1 ]; then cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d \$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 \$GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline $* > \$GRAFT_REPO_ROOT/gpurun_out/bench_$TAG.json 2> \$GRAFT_REPO_ROOT/gpurun_out/bench_$TAG.err; echo prof rc=\$?; fi" > gpurun_out/call_$TAG.txt 2>&1
tail -3 gpurun_out/call_$TAG.txt
tail -4 gpurun_out/pytest_$TAG.log | cut -c1-600
python3 -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], d['verified_bit_exact'], d['roofline']['kernel_ms_avg'], d['path_stats'])" 2>&1 | tail -2
python3 - <<'PY'
import sqlite3, glob
dbs = glob.glob('gpurun_out/prof_$TAG/**/*.db', recursive=True)
if dbs:
    c = sqlite3.connect(dbs[0])
    for r in c.execute("select name,total_calls,average/1e3,percentage from top_kernels limit 6"): print(r[0][:40], r[1], round(r[2],2), 'ms', round(r[3],1))
PY
