#!/bin/bash
# Lane limit 512 KiB with binary-searched group ends: lane tests, size sweep, echo / session legs A/B against $WSG_LANE_MAX=65536 (round 5's limit)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5s}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lane.py > "$OUT/lane_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/lane_tests.log"; exit 1; }
tail -1 "$OUT/lane_tests.log"
timeout -k 10 300 python -u tools/lane_ab.py sweep 600 > "$OUT/lane_sweep.log" 2>&1 || { echo "sweep rc=$?"; tail -20 "$OUT/lane_sweep.log"; exit 1; }
: > "$OUT/ab.log"
for round in 1 2; do
  for lm in default 65536; do
    if [ "$lm" = default ]; then unset WSG_LANE_MAX; else export WSG_LANE_MAX=$lm; fi
    for leg in "bench_echo_tcp gpu_tick 100 4" "bench_echo_tcp gpu 100 4" "bench_echo tick 100 1" "bench_echo per_read 1 1"; do
      set -- $leg
      exe=$1; shift
      r=$(timeout -k 10 60 tools/_build/$exe "$@" 1000 32 2 2>&1 | tail -1) || { echo "fail $leg"; exit 1; }
      echo "lane_max=$lm $leg $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["msg_per_s"], d["payload_ok"])')" >> "$OUT/ab.log"
    done
    for m in rx tx; do
      r=$(timeout -k 10 120 tools/_build/bench_batch $m 256 64 32 0 3 2>&1 | tail -1) || { echo "fail batch $m"; exit 1; }
      echo "lane_max=$lm bench_batch $m 32B $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["batched_frames_per_s"], d["delivered_ok"])')" >> "$OUT/ab.log"
    done
  done
done
unset WSG_LANE_MAX
cat "$OUT/ab.log"
