# round 4: stream kernel in-kernel counters after the window changes (profiling build, batch path)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4k2
mkdir -p $O
cd $R
ZS_STREAM_PK=0 ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_prof.so timeout -k 10 200 python3 -u tools/stream_probe.py 16 32 > $O/one.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/one.txt
