#!/bin/bash
# Copy shapes at C2's size (tools/membench.hip tail): 16 KiB tiles vs 4 KiB tiles (one chunk per lane) for the last pct % or all of the bytes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5k}
mkdir -p "$OUT"
timeout -k 10 200 tools/_build/membench 256 tail > "$OUT/tail_256.log" 2>&1 || { echo "tail rc=$?"; tail "$OUT/tail_256.log"; exit 1; }
cat "$OUT/tail_256.log"
