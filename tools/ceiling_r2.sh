#!/bin/bash
# Round-2 evidence for the C2 ceiling, one GPU call (profiles/r2/ceiling_c2.log):
# k_decode through the C-ABI against a bare copy-with-XOR of the same bytes in
# one process (tools/decbench.hip), membench's copy grid sweep at C2's
# footprint, and bench.py's headline line at 20 and 200 steps on the same box.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ceiling
mkdir -p "$OUT"
{
  echo "== decbench (C2: 4096 x 64 KiB, C++ launch loop, NULL stream)"
  timeout -k 10 120 tools/_build/decbench 4096 65536 cppserver_amd/_build/libwsg.so | grep -v "copy v"
  echo "== membench 256 grid (bare copy vs grid, two buffer pairs)"
  timeout -k 10 120 tools/_build/membench 256 grid
  echo "== bench.py --steps 20"
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-extras | cut -c1-600
  echo "== bench.py --steps 200"
  timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu --no-extras | cut -c1-600
} > "$OUT/ceiling_c2.log" 2>&1
echo done
