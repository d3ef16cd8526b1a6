#!/bin/bash
mkdir -p gpurun_out/dbg
ZS_DEBUG_CHUNKS=2 timeout -k 10 120 python3 tools/dbg/$1.py > gpurun_out/dbg/$1.out 2> gpurun_out/dbg/$1.err; rc=$?
echo rc=$rc
python3 tools/dbg/chain_walk.py gpurun_out/dbg/$1.err
