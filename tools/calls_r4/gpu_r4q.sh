#!/bin/bash
# 100 echo clients on 4 threads: tables in place vs copies, lane profile per context
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4q}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    grep -h "msg_per_s\|WSG_LANE_PROFILE" "$OUT/$name.log" | cut -c1-330
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
step lane_tests 300 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 250 --timeout-method thread
step c100_inplace 60 env WSG_LANE_PROFILE=1 tools/_build/bench_echo per_read 100 4 1000 32 2
step c100_copies 60 env WSG_LANE_PROFILE=1 WSG_TABLES_IN_PLACE=0 tools/_build/bench_echo per_read 100 4 1000 32 2
step c100_nolane 60 env WSG_LANE_MAX=0 tools/_build/bench_echo per_read 100 4 1000 32 2
step c1_inplace 60 env WSG_LANE_PROFILE=1 tools/_build/bench_echo per_read 1 1 1000 32 2
step c1_copies 60 env WSG_LANE_PROFILE=1 WSG_TABLES_IN_PLACE=0 tools/_build/bench_echo per_read 1 1 1000 32 2
step c100_t1 60 env WSG_LANE_PROFILE=1 tools/_build/bench_echo per_read 100 1 1000 32 2
echo "== done"
