#!/bin/bash
# The two sequences that each crashed once (r4s, r4ab), repeated with host backtrace handlers
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4ad}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
    local name=$1
    shift
    WSG_CRASH_TRACE=1 timeout -k 10 60 "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    if [ $rc -ne 0 ]; then tail -45 "$OUT/$name.log"; exit $rc; fi
}
for i in 1 2 3 4 5; do
    run s_c1_$i env WSG_LANE_REQS=1000000 tools/_build/bench_echo_samp per_read 1 1 1000 32 2
    run s_c100_$i env WSG_LANE_REQS=1000000 tools/_build/bench_echo_samp per_read 100 4 1000 32 2
    run t_r32_$i env WSG_LANE_REQS=32 tools/_build/bench_echo_tcp_dbg gpu 100 4 1000 32 2
    run t_idle_$i env WSG_LANE_IDLE_US=100 tools/_build/bench_echo_tcp_dbg gpu 100 4 1000 32 2
done
