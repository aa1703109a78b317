#!/bin/bash
# Lane cap from GPU_MAX_HW_QUEUES: TCP / in-memory echo checks, lane tests, then the driver's line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4an}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $(python -c "import json; print(json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1])['msg_per_s'])" 2>/dev/null)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
    return 0
}
step lane_tests 300 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 250 --timeout-method thread
tail -1 "$OUT/lane_tests.log"
step tcp_hwq8_a 60 env GPU_MAX_HW_QUEUES=8 tools/_build/bench_echo_tcp gpu 100 4 1000 32 2
step tcp_hwq8_b 60 env GPU_MAX_HW_QUEUES=8 tools/_build/bench_echo_tcp gpu 100 4 1000 32 2
step tcp_hwq8_1c 60 env GPU_MAX_HW_QUEUES=8 tools/_build/bench_echo_tcp gpu 1 1 1000 32 2
step tcp_hwq8_tick 60 env GPU_MAX_HW_QUEUES=8 tools/_build/bench_echo_tcp gpu_tick 100 4 1000 32 2
step mem_hwq8_1c 60 env GPU_MAX_HW_QUEUES=8 tools/_build/bench_echo per_read 1 1 1000 32 2
step mem_hwq8_100c 60 env GPU_MAX_HW_QUEUES=8 tools/_build/bench_echo per_read 100 4 1000 32 2
echo "== bench $(date +%T)"
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > "$OUT/bench.out" 2> "$OUT/bench.err" || exit $?
echo "bench done $(date +%T)"
