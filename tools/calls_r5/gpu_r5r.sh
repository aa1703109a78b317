#!/bin/bash
# Lane requests up to 2 MiB in byte-balanced groups: lane tests, lane vs launch path per batch size, echo / session legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5r}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lane.py > "$OUT/lane_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/lane_tests.log"; exit 1; }
tail -1 "$OUT/lane_tests.log"
timeout -k 10 300 python -u tools/lane_ab.py sweep 1000 > "$OUT/lane_sweep.log" 2>&1 || { echo "sweep rc=$?"; tail -20 "$OUT/lane_sweep.log"; exit 1; }
cat "$OUT/lane_sweep.log"
: > "$OUT/echo.log"
for leg in "bench_echo_tcp gpu 100 4" "bench_echo_tcp gpu_tick 100 4" "bench_echo tick 100 1" "bench_echo per_read 1 1" "bench_echo per_read 100 4"; do
  set -- $leg
  exe=$1; shift
  r=$(timeout -k 10 60 tools/_build/$exe "$@" 1000 32 2 2>&1 | tail -1) || { echo "fail $leg"; exit 1; }
  echo "$leg $r" >> "$OUT/echo.log"
done
for m in rx tx; do
  timeout -k 10 120 tools/_build/bench_batch $m 256 64 32 0 3 >> "$OUT/echo.log" 2>&1 || { echo "fail batch $m"; exit 1; }
done
cat "$OUT/echo.log"
