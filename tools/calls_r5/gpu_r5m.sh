#!/bin/bash
# Parallel staging copies: worker count A/B on the host-staged C2 decode / encode (tools/pcie_pageable.py), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5m}
mkdir -p "$OUT"
: > "$OUT/copy_workers_ab.log"
for round in 1 2 3; do
  for n in 1 3 5 7 11; do
    timeout -k 10 120 python tools/pcie_pageable.py cppserver_amd/_build/var/cw$n/libwsg.so 2>/dev/null | tail -1 | sed "s/^/workers=$n /" >> "$OUT/copy_workers_ab.log" || { echo "cw$n failed"; exit 1; }
  done
done
cat "$OUT/copy_workers_ab.log"
