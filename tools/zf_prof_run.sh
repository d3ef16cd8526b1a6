mkdir -p gpurun_out/zfp
ZS_LIB=$GRAFT_REPO_ROOT/zlib-streams_amd/libzstreams_mi355x_zfprof.so timeout -k 10 200 python3 -u -c "
import sys; sys.path.insert(0,'zlib-streams_amd'); sys.path.insert(0,'tests')
import corpus, zstreams
for sid in (0, 33):
    d = corpus.stream(sid, 4 << 20)
    for lv in (1, 3):
        zstreams.deflate_batch([d], -15, lv)
" > gpurun_out/zfp/out.log 2>&1; echo rc=$?; cat gpurun_out/zfp/out.log
