#!/bin/bash
# Status from the latch on the staged pipeline too: lane tests (latch cases), then host decode times product vs the pre-latch library (var/no_latch), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5y}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lane.py > "$OUT/tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
: > "$OUT/ab.log"
for round in 1 2; do
  for lib in - cppserver_amd/_build/var/no_latch/libwsg.so; do
    timeout -k 10 300 python -u tools/latch_ab.py $lib 20 >> "$OUT/ab.log" 2>&1 || { echo "ab rc=$?"; tail -5 "$OUT/ab.log"; exit 1; }
  done
done
grep '^{' "$OUT/ab.log"
