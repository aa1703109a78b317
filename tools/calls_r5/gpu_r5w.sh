#!/bin/bash
# Kernel times of tick-sized host batches read in place over PCIe (100000 x 38 B, 3.8 MB; 16384 x 38 B, 622 KB): rocprofv3 kernel trace of tools/lane_ab.py
# (the echo binaries call wsg_destroy from thread-exit destructors, which rocprofv3 3.x aborts on)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5w}
mkdir -p "$OUT"
export TMPDIR=/tmp
for shape in "100000 32" "16384 32"; do
  tag=${shape// /_}
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/p_$tag" -o run -- python3 tools/lane_ab.py $shape 200 > "$OUT/lane_ab_$tag.log" 2>&1 || { echo "prof $shape rc=$?"; grep -v simple_timer "$OUT/lane_ab_$tag.log" | tail -8; exit 1; }
  grep '^{' "$OUT/lane_ab_$tag.log"
done
find "$OUT" -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-8 "$f" | head -8; done
