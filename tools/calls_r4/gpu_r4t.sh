#!/bin/bash
# The 100-client echo that crashed once (rc 139, r4s): repeated with a host backtrace handler
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4t}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
  for r in 1000000; do
    echo "== run $i reqs $r $(date +%T)"
    WSG_CRASH_TRACE=1 WSG_LANE_REQS=$r timeout -k 10 60 tools/_build/bench_echo_samp per_read 100 4 1000 32 2 > "$OUT/c100_${r}_$i.log" 2>&1
    rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -40 "$OUT/c100_${r}_$i.log"; exit $rc; fi
    tail -1 "$OUT/c100_${r}_$i.log" | cut -c1-200
  done
done
