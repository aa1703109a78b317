#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4g}
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
step echo_lane_profile 120 env WSG_LANE_PROFILE=1 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
step slide_parity 300 python -u tools/variant_parity.py fan_slide 120 --fanout
step slide_parity_w3 300 env WSG_FAN_WAVES_PER_CU=3 python -u tools/variant_parity.py fan_slide 60 --fanout
step fan_slide_ab 300 python -u tools/fan_many_ab.py "" "lib:fan_slide" "lib:fan_slide,WSG_FAN_WAVES_PER_CU=4" "lib:fan_slide,WSG_FAN_WAVES_PER_CU=3" "lib:fan_slide,WSG_FAN_WAVES_PER_CU=2" "lib:fan_slide,WSG_FAN_WAVES_PER_CU=5"
echo "== done"
