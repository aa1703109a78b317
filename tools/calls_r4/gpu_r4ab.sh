#!/bin/bash
# Many lanes at once (TCP echo: 4 server + 4 client threads): workgroups per lane, hand-over period
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $(python -c "import json; print(json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1])['msg_per_s'])" 2>/dev/null)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
for w in 1 2 4; do
step tcp_100c_w$w 60 env WSG_LANE_WGS=$w tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
step tcp_tick_w$w 60 env WSG_LANE_WGS=$w tools/_build/bench_echo_tcp gpu_tick 100 4 1000 32 3
step mem_100c_w$w 60 env WSG_LANE_WGS=$w tools/_build/bench_echo per_read 100 4 1000 32 3
done
step tcp_100c_r32 60 env WSG_LANE_REQS=32 tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
step tcp_100c_idle100 60 env WSG_LANE_IDLE_US=100 tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
step tcp_tick_idle100 60 env WSG_LANE_IDLE_US=100 tools/_build/bench_echo_tcp gpu_tick 100 4 1000 32 3
step tcp_100c_lanemax8k 60 env WSG_LANE_MAX=8192 tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
echo "== done"
