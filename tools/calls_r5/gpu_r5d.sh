#!/bin/bash
# Write-run patterns (tools/membench.hip wrun): U contiguous rows per wave vs the fill, 16-message tick and one C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5d}
mkdir -p "$OUT"
timeout -k 10 120 tools/_build/membench 626 wrun > "$OUT/wrun_626.log" 2>&1 || { echo "wrun 626 rc=$?"; tail "$OUT/wrun_626.log"; exit 1; }
cat "$OUT/wrun_626.log"
timeout -k 10 120 tools/_build/membench 0 wrun > "$OUT/wrun_c4.log" 2>&1 || { echo "wrun c4 rc=$?"; tail "$OUT/wrun_c4.log"; exit 1; }
cat "$OUT/wrun_c4.log"
