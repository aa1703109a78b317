#!/bin/bash
# Lanes on high-priority streams vs the default priority: TCP echo (launch-path reads next to lanes) and in-memory echo
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4aa}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    grep -h "msg_per_s" "$OUT/$name.log" | cut -c1-200
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
for p in 1 0; do
step tcp_100c_p$p 60 env WSG_LANE_PRIORITY=$p tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
step tcp_tick_p$p 60 env WSG_LANE_PRIORITY=$p tools/_build/bench_echo_tcp gpu_tick 100 4 1000 32 3
step tcp_1c_p$p 60 env WSG_LANE_PRIORITY=$p tools/_build/bench_echo_tcp gpu 1 1 1000 32 3
step mem_100c_p$p 60 env WSG_LANE_PRIORITY=$p tools/_build/bench_echo per_read 100 4 1000 32 3
step mem_1c_p$p 60 env WSG_LANE_PRIORITY=$p tools/_build/bench_echo per_read 1 1 1000 32 3
done
step tcp_tick_nolane 60 env WSG_LANE_MAX=0 tools/_build/bench_echo_tcp gpu_tick 100 4 1000 32 3
step tcp_100c_nolane 60 env WSG_LANE_MAX=0 tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
echo "== done"
