#!/bin/bash
# Baseline at the start of round 5: TCP echo (default env) and the per-call path
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5a}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 60 "$@" > "$OUT/$name.log" 2>&1 || { echo "$name rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }; echo "$name $(tail -1 "$OUT/$name.log" | cut -c1-160)"; }
run tcp_gpu_1c tools/_build/bench_echo_tcp gpu 1 1 1000 32 3
run tcp_gpu_100c tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
run tcp_ref_100c tools/_build/bench_echo_tcp cpu_ref 100 4 1000 32 3
run mem_per_call tools/_build/bench_echo per_call 1 1 1000 32 3
run mem_per_read tools/_build/bench_echo per_read 1 1 1000 32 3
run mem_per_read_100c tools/_build/bench_echo per_read 100 4 1000 32 3
