#!/bin/bash
# The TCP echo that crashed with a 100 us lane idle limit (r4ab): repeated with a host backtrace handler
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4ac}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
    WSG_CRASH_TRACE=1 WSG_LANE_IDLE_US=100 timeout -k 10 60 tools/_build/bench_echo_tcp_dbg gpu 100 4 1000 32 2 > "$OUT/run$i.log" 2>&1
    rc=$?
    echo "run $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -45 "$OUT/run$i.log"; exit $rc; fi
done
