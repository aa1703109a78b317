#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4f}
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
step echo_prof_1c 120 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
step echo_prof_100c 120 tools/_build/bench_echo_prof per_read 100 4 1000 32 3
step host_suites 600 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_rx_batch.py tests/test_gpu_tx_batch.py tests/test_gpu_cpp_api.py tests/test_gpu_session.py tests/test_gpu_host_multi.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
echo "== done"
