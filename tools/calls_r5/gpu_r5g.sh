#!/bin/bash
# Lane workgroup count A/B ($WSG_LANE_WGS 4 / 8 / 16) on the echo legs, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5g}
mkdir -p "$OUT"
: > "$OUT/wgs_ab.log"
for round in 1 2; do
  for w in 4 8 16; do
    for leg in "bench_echo per_read 1 1" "bench_echo per_read 100 4" "bench_echo per_call 1 1" "bench_echo_tcp gpu 100 4" "bench_echo_tcp gpu 1 1"; do
      set -- $leg
      exe=$1; shift
      r=$(WSG_LANE_WGS=$w timeout -k 10 60 tools/_build/$exe "$@" 1000 32 2 2>&1 | tail -1) || { echo "fail $w $leg"; exit 1; }
      echo "wgs=$w $leg $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["msg_per_s"], d["payload_ok"])')" | tee -a "$OUT/wgs_ab.log"
    done
  done
done
