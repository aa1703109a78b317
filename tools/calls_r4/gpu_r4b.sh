#!/bin/bash
# Round 4, second GPU call: the whole GPU suite on the new host paths, the
# small-pass latency micro-benchmark (C1), the fan-out store-policy A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4b}
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
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smallpass_38k 120 tools/_build/smallpass 38000 2000
step smallpass_4k 120 tools/_build/smallpass 4000 2000
step fan_many_ab 240 python -u tools/fan_many_ab.py "" lib:fan_nt lib:fan_aux0 lib:fan_aux17 lib:fan_unroll2 "WSG_FAN_WAVES_PER_CU=8,WSG_FAN_WPB=8"
echo "== done"
