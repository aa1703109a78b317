#!/bin/bash
# TCP echo 100 clients on 4+4 threads: hardware queues per process (GPU_MAX_HW_QUEUES) x lanes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4am}
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
for q in 4 8 16; do
  step tcp_q${q}_cap4 60 env GPU_MAX_HW_QUEUES=$q tools/_build/bench_echo_tcp gpu 100 4 1000 32 2
  step tcp_q${q}_cap8 60 env GPU_MAX_HW_QUEUES=$q WSG_LANE_CAP=8 tools/_build/bench_echo_tcp gpu 100 4 1000 32 2
  step tcp_q${q}_nolane 60 env GPU_MAX_HW_QUEUES=$q WSG_LANE_MAX=0 tools/_build/bench_echo_tcp gpu 100 4 1000 32 2
  step mem_q${q}_100c 60 env GPU_MAX_HW_QUEUES=$q tools/_build/bench_echo per_read 100 4 1000 32 2
done
echo "== done"
