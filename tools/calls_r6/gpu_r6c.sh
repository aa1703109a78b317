#!/bin/bash
# Debug of the lane's launch count in the ticket-wrap job: per-call XORs with
# and without the ticket-base hook, lane stats along the way.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6c}
mkdir -p "$OUT"
timeout -k 10 60 python -u tools/wrap_dbg.py > "$OUT/plain.log" 2>&1 || { echo "plain rc=$?"; cat "$OUT/plain.log"; exit 1; }
WSG_TEST_LANE_TICKET_BASE=$((2**32-300)) timeout -k 10 60 python -u tools/wrap_dbg.py > "$OUT/base.log" 2>&1 || { echo "base rc=$?"; cat "$OUT/base.log"; exit 1; }
WSG_TEST_LANE_TICKET_BASE=$((2**32-300)) WSG_TEST_LANE_STALE_XRES=1 timeout -k 10 60 python -u tools/wrap_dbg.py > "$OUT/stale.log" 2>&1 || { echo "stale rc=$?"; cat "$OUT/stale.log"; exit 1; }
tail -n 4 "$OUT/plain.log" "$OUT/base.log" "$OUT/stale.log"
