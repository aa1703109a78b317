#!/bin/bash
# Round 4: the host lane — its tests, the fuzz suites of the host paths, the
# C1 echo with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4c}
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
step host_suites 600 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_rx_batch.py tests/test_gpu_tx_batch.py tests/test_gpu_cpp_api.py tests/test_gpu_session.py tests/test_gpu_host_multi.py -x -q --timeout 300 --timeout-method thread
step echo_prof_1c 120 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
step echo_prof_1c_nolane 120 env WSG_LANE_MAX=0 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
step echo_prof_100c 120 tools/_build/bench_echo_prof per_read 100 4 1000 32 3
step echo_tick_100c 120 tools/_build/bench_echo tick 100 1 1000 32 3
step echo_ref_1c 120 tools/_build/bench_echo_ref 1 1 1000 32 3
step echo_ref_100c 120 tools/_build/bench_echo_ref 100 4 1000 32 3
step edge2_parity 300 python -u tools/variant_parity.py edge2 300
step edge2_diag 300 python -u tools/c3_enc_diag.py edge2 diag4
step membench_wpattern 200 tools/_build/membench 626 wpattern
step membench_write 200 tools/_build/membench 626 write
echo "== done"
