# round 4: zlib-bytes tree kernel phase clocks on the stream surface (random / lines L6)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4u
mkdir -p $O
cd $R
for K in random lines; do
ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_treeprof.so LEVELS=6 KINDS=$K timeout -k 10 200 python3 -u tools/dstream_probe.py 1 > $O/tree_$K.log 2>&1 || exit $?
grep "zd_tree" $O/tree_$K.log | head -8; grep GPU $O/tree_$K.log
done
