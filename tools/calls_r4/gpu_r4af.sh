#!/bin/bash
# The crash of r4ae (one lane, three launch-path contexts, in-memory echo 100c/4t) with a host backtrace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4af}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3 4 5 6 7 8; do
    WSG_CRASH_TRACE=1 WSG_LANE_CAP=1 timeout -k 10 60 tools/_build/bench_echo_samp per_read 100 4 1000 32 2 > "$OUT/run$i.log" 2>&1
    rc=$?
    echo "run $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -45 "$OUT/run$i.log"; exit $rc; fi
done
