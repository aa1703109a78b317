#!/bin/bash
# TCP echo 100 clients on 4+4 threads, sampled with call stacks (where the host time goes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4al}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_SAMPLER=200 WSG_SAMPLER_STACKS=1 WSG_SAMPLER_OUT=$OUT/tcp100.txt timeout -k 10 60 tools/_build/bench_echo_tcp_dbg gpu 100 4 1000 32 3 > "$OUT/tcp100.log" 2>&1 || exit $?
tail -1 "$OUT/tcp100.log" | cut -c1-200
WSG_SAMPLER=200 WSG_SAMPLER_STACKS=1 WSG_SAMPLER_OUT=$OUT/tcp100_nolane.txt WSG_LANE_MAX=0 timeout -k 10 60 tools/_build/bench_echo_tcp_dbg gpu 100 4 1000 32 3 > "$OUT/tcp100_nolane.log" 2>&1 || exit $?
tail -1 "$OUT/tcp100_nolane.log" | cut -c1-200
