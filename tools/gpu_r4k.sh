# round 4: in-kernel counters, one handle vs 64 handles (profiling build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4k
mkdir -p $O
cd $R
export ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_prof.so
timeout -k 10 200 python3 -u tools/stream_probe.py 16 32 > $O/one.txt 2>&1 || exit $?
cat $O/one.txt | grep -v amdgpu.ids
for NH in 8 64; do
ZS_STREAM_SLOTS=1 ZS_STREAM_GATHER_US=200 timeout -k 10 200 python3 -u tools/stream_agg_probe.py $NH 4 > $O/agg$NH.txt 2>&1 || exit $?
echo "== $NH handles"; cat $O/agg$NH.txt | grep -v amdgpu.ids
done
