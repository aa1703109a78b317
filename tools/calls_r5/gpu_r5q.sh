#!/bin/bash
# TCP echo 100c/4t at the default environment, repeated, with the lane counters; one launch-path-only run for comparison
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5q}
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/tcp_repeat.log"
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 60 tools/_build/bench_echo_tcp gpu 100 4 1000 32 2 >> "$OUT/tcp_repeat.log" 2>&1 || { echo "fail run $i"; tail -5 "$OUT/tcp_repeat.log"; exit 1; }
done
WSG_LANE_MAX=0 timeout -k 10 60 tools/_build/bench_echo_tcp gpu 100 4 1000 32 2 >> "$OUT/tcp_repeat.log" 2>&1 || { echo "fail launch-only"; exit 1; }
cat "$OUT/tcp_repeat.log"
