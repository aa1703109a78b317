#!/bin/bash
# After the spin queue lock, initial-exec TLS and the warmed codec: API tests, echo 1c / 100c vs the reference loop
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4v}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    grep -h "msg_per_s\|passed\|failed" "$OUT/$name.log" | cut -c1-250
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
step api_tests 400 python -u -m pytest tests/test_gpu_cpp_api.py tests/test_gpu_tx_batch.py tests/test_gpu_rx_batch.py tests/test_gpu_session.py tests/test_gpu_lane.py -x -q --timeout 300 --timeout-method thread
for i in 1 2; do
step echo_1c_$i 60 tools/_build/bench_echo per_read 1 1 1000 32 3
step ref_1c_$i 60 tools/_build/bench_echo_ref -c 1 -t 1 -m 1000 -s 32 -z 3
done
step hostonly_1c 60 tools/_build/echo_hostonly per_read 1 1 1000 32 3
step echo_100c 60 tools/_build/bench_echo per_read 100 4 1000 32 3
step ref_100c 60 tools/_build/bench_echo_ref -c 100 -t 4 -m 1000 -s 32 -z 3
step echo_tick_100c 60 tools/_build/bench_echo tick 100 1 1000 32 3
step samp_1c 60 env WSG_SAMPLER=100 WSG_SAMPLER_STACKS=1 WSG_SAMPLER_OUT=$OUT/samp_1c.txt tools/_build/bench_echo_samp per_read 1 1 1000 32 3
echo "== done"
