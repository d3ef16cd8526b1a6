#!/bin/bash
# Round-2 first GPU check: host facts, GPU parity tests, short inflate bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2a
mkdir -p $O
cd $R
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -E "Model name|Socket|Core|Thread|^CPU\(s\)"; python3 -c "import os;print('affinity',len(os.sched_getaffinity(0)))"; free -g | head -2; } > $O/host.txt 2>&1
cat $O/host.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -8 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline --no-compress --no-deflate64 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json
exit $rc
