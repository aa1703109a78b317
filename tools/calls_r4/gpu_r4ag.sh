#!/bin/bash
# The driver's command under rocprofv3 --kernel-trace --marker-trace --stats (host legs skipped: their child processes' launches take minutes to trace)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/art_r4
mkdir -p "$OUT"
export TMPDIR=/tmp
export WSG_BENCH_HOST_LEGS=0
echo "== trace $(date +%T)"
timeout -k 10 900 rocprofv3 --kernel-trace --marker-trace --stats -d "$OUT/trace" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 > "$OUT/trace.out" 2> "$OUT/trace.err"
rc=$?
echo "rc=$rc $(date +%T)"
tail -c 400 "$OUT/trace.out"
exit $rc
