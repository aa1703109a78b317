#!/bin/bash
# Round 4: the lane after the relaxed poll; where its time goes (timing-only
# builds); the lane tests; the echo.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4d}
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
step lane_tests 300 python -u -m pytest tests/test_gpu_lane.py -x -v --timeout 250 --timeout-method thread
step lane_ab 300 python -u tools/lane_ab.py
step lane_ab_4k 300 python -u tools/lane_ab.py 100 32 3000
step echo_prof_1c 120 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
echo "== done"
