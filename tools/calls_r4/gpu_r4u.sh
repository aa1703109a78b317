#!/bin/bash
# Sampled echo at 1 client with call stacks (what the host does besides the codec)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4u}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_SAMPLER=100 WSG_SAMPLER_STACKS=1 WSG_SAMPLER_OUT=$OUT/samp_1c.txt timeout -k 10 60 tools/_build/bench_echo_samp per_read 1 1 1000 32 4 > "$OUT/samp_1c.log" 2>&1 || exit $?
tail -1 "$OUT/samp_1c.log"
WSG_SAMPLER=100 WSG_SAMPLER_STACKS=1 WSG_SAMPLER_OUT=$OUT/samp_1c_reqs1m.txt WSG_LANE_REQS=1000000 timeout -k 10 60 tools/_build/bench_echo_samp per_read 1 1 1000 32 4 > "$OUT/samp_1c_reqs1m.log" 2>&1 || exit $?
tail -1 "$OUT/samp_1c_reqs1m.log"
