# round 4: deflate_fast kernel phase clocks (profiling variant), one handle L1 lines 1 MiB
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s
mkdir -p $O
cd $R
ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_zfprof.so LEVELS=1 KINDS=lines timeout -k 10 200 python3 -u tools/dstream_probe.py 1 > $O/zf.log 2>&1; rc=$?
echo rc=$rc; grep -c "zf job" $O/zf.log; grep "zf job" $O/zf.log | head -12; grep GPU $O/zf.log
