# round 4: stream window change -- inflate + stream tests, stream leg, in-kernel phase counters
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4z5
mkdir -p $O
cd $R
bash tools/gpu_r4x.sh || exit $?
ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_prof.so timeout -k 10 200 python3 tools/stream_probe.py 16 > $O/probe_prof.log 2>&1; rc=$?
tail -3 $O/probe_prof.log; exit $rc
