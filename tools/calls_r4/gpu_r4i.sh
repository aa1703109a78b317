#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4i}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
step lane_tests 300 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 250 --timeout-method thread
step echo_profile 120 env WSG_LANE_PROFILE=1 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
step echo_100c 120 tools/_build/bench_echo_prof per_read 100 4 1000 32 3
step lane_ab 300 python -u tools/lane_ab.py
echo "== done"
