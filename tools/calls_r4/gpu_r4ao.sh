#!/bin/bash
# Final tree: 2000-seed differential fuzz (encode/decode, host pair, fan-out), then the driver's command under rocprofv3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/art_r4
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== fuzz $(date +%T)"
WSG_FUZZ_SEEDS=2000 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > "$OUT/fuzz2000.log" 2>&1
rc=$?
tail -2 "$OUT/fuzz2000.log"
[ $rc -ne 0 ] && exit $rc
echo "== trace $(date +%T)"
WSG_BENCH_HOST_LEGS=0 timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace --stats -d "$OUT/trace" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 > "$OUT/trace.out" 2> "$OUT/trace.err"
rc=$?
echo "rc=$rc $(date +%T)"
exit $rc
