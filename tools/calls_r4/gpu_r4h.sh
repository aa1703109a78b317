#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4h}
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
step echo_default 120 env WSG_LANE_PROFILE=1 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
step echo_coherent 120 env WSG_LANE_PROFILE=1 WSG_HOST_COHERENT=1 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
step echo_coherent_nolane 120 env WSG_HOST_COHERENT=1 WSG_LANE_MAX=0 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
step echo_coherent_100c 120 env WSG_HOST_COHERENT=1 tools/_build/bench_echo_prof per_read 100 4 1000 32 3
step lane_tests_coherent 300 env WSG_HOST_COHERENT=1 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_rx_batch.py tests/test_gpu_tx_batch.py -x -q --timeout 250 --timeout-method thread
step batch_coherent 200 env WSG_HOST_COHERENT=1 tools/_build/bench_batch rx 1024 4 65536 16384 3
step batch_default 200 tools/_build/bench_batch rx 1024 4 65536 16384 3
echo "== done"
