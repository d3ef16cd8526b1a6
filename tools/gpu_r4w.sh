# round 4: msearch walk donation A/B (variant library) on the 16 x 64 MiB zlib-bytes batch
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for V in ${VARS:-base donate}; do
  if [ $V = base ]; then unset ZS_LIB; else export ZS_LIB=$R/zlib-streams_amd/libzstreams_mi355x_$V.so; fi
  timeout -k 10 300 python3 tools/zd_probe.py 2>&1 | grep "zlib-bytes" | sed "s/^/$V /" || exit 1
  timeout -k 10 300 python3 tools/zd_probe.py --level 9 --streams 8 2>&1 | grep "zlib-bytes" | sed "s/^/$V /" || exit 1
done
