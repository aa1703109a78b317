#!/bin/bash
# Lane yield interval A/B ($WSG_LANE_YIELD_US 500 / 2000 / 8000) on the echo legs, interleaved; then the full GPU suite and smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5n}
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/yield_ab.log"
for round in 1 2; do
  for y in 500 2000 8000; do
    for leg in "bench_echo per_read 1 1" "bench_echo per_read 100 4" "bench_echo_tcp gpu 100 4"; do
      set -- $leg
      exe=$1; shift
      r=$(WSG_LANE_YIELD_US=$y timeout -k 10 60 tools/_build/$exe "$@" 1000 32 2 2>&1 | tail -1) || { echo "fail $y $leg"; exit 1; }
      echo "yield_us=$y $leg $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["msg_per_s"], d["payload_ok"])')" | tee -a "$OUT/yield_ab.log"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu suite rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
