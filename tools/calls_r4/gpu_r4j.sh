#!/bin/bash
# Round 4: host path after the batch changes (announce on change, one
# SendAsync per run, scope sends without the connection's send lock) and the
# host lane; the echo at 1c / 100c next to the host-only and reference loops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4j}
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
step api_tests 400 python -u -m pytest tests/test_gpu_cpp_api.py tests/test_gpu_tx_batch.py tests/test_gpu_rx_batch.py tests/test_gpu_session.py tests/test_gpu_lane.py -x -q --timeout 300 --timeout-method thread
for i in 1 2; do
step echo_1c_$i 60 tools/_build/bench_echo per_read 1 1 1000 32 3
step hostonly_1c_$i 60 tools/_build/echo_hostonly per_read 1 1 1000 32 3
step ref_1c_$i 60 tools/_build/bench_echo_ref -c 1 -t 1 -m 1000 -s 32 -z 3
done
step echo_100c 60 tools/_build/bench_echo per_read 100 4 1000 32 3
step ref_100c 60 tools/_build/bench_echo_ref -c 100 -t 4 -m 1000 -s 32 -z 3
step echo_profile 60 env WSG_LANE_PROFILE=1 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
echo "== done"
