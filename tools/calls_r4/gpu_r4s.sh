#!/bin/bash
# Lane hand-over period vs the echo at 1 client and 100 clients / 4 threads; sampled at 1 client
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4s}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    grep -h "msg_per_s" "$OUT/$name.log" | cut -c1-250
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
for r in 16 256 4096 1000000; do
step c1_reqs$r 60 env WSG_LANE_REQS=$r tools/_build/bench_echo per_read 1 1 1000 32 2
step c100_reqs$r 60 env WSG_LANE_REQS=$r tools/_build/bench_echo per_read 100 4 1000 32 2
done
step samp_reqs1000000 60 env WSG_LANE_REQS=1000000 WSG_SAMPLER=100 WSG_SAMPLER_OUT=$OUT/samp_1c_noho.txt tools/_build/bench_echo_samp per_read 1 1 1000 32 4
echo "== done"
