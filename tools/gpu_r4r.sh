# round 4: deflate stream surface per-kernel profile (L6 random = the reference perf workload shape, L1 lines)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for CFG in "6 random" "1 lines" "6 lines"; do
  set -- $CFG
  LEVELS=$1 KINDS=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$1_$2 -o run -- python3 $R/tools/dstream_probe.py 4 > $O/probe_$1_$2.log 2>&1 || exit $?
  grep -v amdgpu.ids $O/probe_$1_$2.log
  f=$(find $O/prof_$1_$2 -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 $f | head -14
  find $O/prof_$1_$2 -name "*kernel_trace.csv" -delete
done
