#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4e}
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
step lane_ab 300 python -u tools/lane_ab.py
step lane_ab_4k 300 python -u tools/lane_ab.py 100 32 3000
step smallpass_38k 120 tools/_build/smallpass 38000 2000
step fan_kv 300 python -u tools/fan_many_ab.py "" "lib:fan_kv4,WSG_FAN_WAVES_PER_CU=4" "lib:fan_kv4,WSG_FAN_WAVES_PER_CU=3" "lib:fan_kv4,WSG_FAN_WAVES_PER_CU=5" "lib:fan_kv3,WSG_FAN_WAVES_PER_CU=4" "WSG_FAN_WAVES_PER_CU=5" "lib:fan_kv4"
echo "== done"
