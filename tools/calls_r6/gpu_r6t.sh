#!/bin/bash
# Pageable host-inclusive C2 decode by NUMA binding of the calling process
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6t}
mkdir -p "$OUT"
: > "$OUT/pageable_numa.log"
for round in 1 2 3; do
  for m in none gpu other; do
    timeout -k 10 120 python tools/pageable_numa.py $m >> "$OUT/pageable_numa.log" 2>&1 || { echo "rc=$? $m"; tail -5 "$OUT/pageable_numa.log"; exit 1; }
  done
done
grep '^{' "$OUT/pageable_numa.log"
