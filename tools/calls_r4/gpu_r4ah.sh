#!/bin/bash
# TCP echo 100 clients on 4+4 threads: lane profile per context, calls timed by the interposer
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4ah}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_LANE_PROFILE=1 timeout -k 10 60 tools/_build/bench_echo_tcp gpu 100 4 1000 32 2 > "$OUT/tcp_lane_prof.log" 2>&1 || exit $?
grep -h "WSG_LANE_PROFILE\|msg_per_s" "$OUT/tcp_lane_prof.log" | cut -c1-330
WSG_LANE_PROFILE=1 WSG_LANE_CAP=1000 timeout -k 10 60 tools/_build/bench_echo_tcp gpu 100 4 1000 32 2 > "$OUT/tcp_lane_prof_all.log" 2>&1 || exit $?
grep -h "WSG_LANE_PROFILE\|msg_per_s" "$OUT/tcp_lane_prof_all.log" | cut -c1-330
for i in 1 2 3 4 5 6; do
  timeout -k 10 60 tools/_build/bench_echo_tcp gpu 100 4 1000 32 1 > "$OUT/tcp_rep$i.log" 2>&1 || { tail -30 "$OUT/tcp_rep$i.log"; exit 1; }
  timeout -k 10 60 tools/_build/bench_echo per_read 100 4 1000 32 1 > "$OUT/mem_rep$i.log" 2>&1 || { tail -30 "$OUT/mem_rep$i.log"; exit 1; }
done
echo "repeats ok"
