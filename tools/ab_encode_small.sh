#!/bin/bash
# A/B of the batch-encode kernels on small/mid frame batches (GPU box): the
# default build, the previous commit (head), and the piece kernel
# (WSG_SMALL_AVG=0, listed last: tune_enc sets each library's env in turn).
# Build the variants first: tools/build_variant.sh pieces (head: the previous commit, built from a git worktree)
mkdir -p gpurun_out/ab
V=cppserver_amd/_build/var
for spec in "1000000 32 32" "1000000 0 64" "200000 0 1024" "50000 0 4096" "20000 0 8192"; do set -- $spec
CFG=c3 FRAMES=$1 LO=$2 HI=$3 REPS=5 timeout -k 10 300 python tools/tune_enc.py cppserver_amd/_build/libwsg.so $V/head/libwsg.so WSG_SMALL_AVG=0@$V/pieces/libwsg.so > gpurun_out/ab/t.log 2>&1 || { cat gpurun_out/ab/t.log; exit 1; }
echo "== frames=$1 payload=$2..$3"; grep kernel gpurun_out/ab/t.log | cut -c1-170
done
