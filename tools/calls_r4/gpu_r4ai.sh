#!/bin/bash
# After the env lock and the per-thread pinned-block cache: lane tests, echo modes (lane cap 4 default vs none)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4ai}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $(grep -h 'WSG_LANE_PROFILE' "$OUT/$name.log" | head -2 | cut -c1-120 | tr '\n' ' ') $(python -c "import json; print(json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1])['msg_per_s'])" 2>/dev/null)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$OUT/$name.log"; exit $rc; fi
    return 0
}
step lane_tests 300 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_cpp_api.py -x -q --timeout 250 --timeout-method thread
tail -1 "$OUT/lane_tests.log"
step tcp_100c_prof 60 env WSG_LANE_PROFILE=1 tools/_build/bench_echo_tcp gpu 100 4 1000 32 2
step tcp_100c 60 tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
step tcp_100c_nolane 60 env WSG_LANE_MAX=0 tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
step tcp_tick 60 tools/_build/bench_echo_tcp gpu_tick 100 4 1000 32 3
step tcp_1c 60 tools/_build/bench_echo_tcp gpu 1 1 1000 32 3
step mem_100c 60 tools/_build/bench_echo per_read 100 4 1000 32 3
step mem_1c 60 tools/_build/bench_echo per_read 1 1 1000 32 3
step ref_tcp_100c 60 tools/_build/bench_echo_tcp cpu_ref 100 4 1000 32 3
echo "== done"
