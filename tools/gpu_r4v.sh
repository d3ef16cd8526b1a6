# round 4: zlib-bytes parse pieces of 64 (ZD_PT=1024) vs 256 -- stream surface and the 16 x 64 MiB batch
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4v
mkdir -p $O
cd $R
for V in base pt1024; do
  if [ $V = base ]; then unset ZS_LIB; else export ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_$V.so; fi
  for K in random lines zipf; do
    LEVELS=6 KINDS=$K timeout -k 10 200 python3 -u tools/dstream_probe.py 4 2>&1 | grep GPU | sed "s/^/$V /" || exit 1
  done
  timeout -k 10 300 python3 tools/zd_probe.py 2>&1 | grep "zlib-bytes" | sed "s/^/$V /" || exit 1
done
