#!/bin/bash
# Lane polling its first word only: tests, echo at 1 / 100 clients by workgroup count
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4o}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    tail -1 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
step lane_tests 300 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 250 --timeout-method thread
for w in 1 4 8; do
step echo_1c_w$w 60 env WSG_LANE_WGS=$w tools/_build/bench_echo per_read 1 1 1000 32 2
step echo_100c_w$w 60 env WSG_LANE_WGS=$w tools/_build/bench_echo per_read 100 4 1000 32 2
done
step ref_1c 60 tools/_build/bench_echo_ref -c 1 -t 1 -m 1000 -s 32 -z 2
step ref_100c 60 tools/_build/bench_echo_ref -c 100 -t 4 -m 1000 -s 32 -z 2
step prof_1c 60 env WSG_LANE_PROFILE=1 tools/_build/bench_echo_prof per_read 1 1 1000 32 2
grep WSG_LANE_PROFILE "$OUT/prof_1c.log"
echo "== done"
