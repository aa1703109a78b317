#!/bin/bash
# Lane diagnostic build (WSG_DIAG_LANE: mailbox positions at a give-up) on the
# ticket-base hook: small base and base near 2^32.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6d}
mkdir -p "$OUT"
export WSG_LIB_PATH=$PWD/cppserver_amd/_build/var/diaglane/libwsg.so WSG_LANE_TIMEOUT_MS=300
for b in 1024 4096 $((2**32-300)); do
  WSG_TEST_LANE_TICKET_BASE=$b timeout -k 10 60 python -u tools/wrap_dbg.py > "$OUT/base_$b.log" 2>&1 || { echo "base $b rc=$?"; cat "$OUT/base_$b.log"; exit 1; }
  echo "== base $b"; head -n 14 "$OUT/base_$b.log"; tail -n 1 "$OUT/base_$b.log"
done
