#!/bin/bash
# Shared device lane: lane tests, then the echo legs (TCP default env, per-call, per-read)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lane.py > "$OUT/lane_tests.log" 2>&1 || { echo "lane tests rc=$?"; tail -30 "$OUT/lane_tests.log"; exit 1; }
tail -3 "$OUT/lane_tests.log"
run() { local name=$1; shift; timeout -k 10 60 "$@" > "$OUT/$name.log" 2>&1 || { echo "$name rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }; echo "$name $(tail -1 "$OUT/$name.log" | cut -c1-200)"; }
run mem_per_call tools/_build/bench_echo per_call 1 1 1000 32 3
run mem_per_read tools/_build/bench_echo per_read 1 1 1000 32 3
run mem_per_read_100c tools/_build/bench_echo per_read 100 4 1000 32 3
run tcp_gpu_1c tools/_build/bench_echo_tcp gpu 1 1 1000 32 3
run tcp_gpu_100c tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
run tcp_ref_100c tools/_build/bench_echo_tcp cpu_ref 100 4 1000 32 3
