#!/bin/bash
# Lane task round trip (tools/lane_rtt.cpp, 32 B inline XOR) by workgroup count 1-16, host thread on the GPU's NUMA node
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5ak}
mkdir -p "$OUT"
export TMPDIR=/tmp
CPUS=$(timeout -k 10 120 python3 -c 'import sys; sys.path.insert(0, "."); import bench; n, c = bench.gpu_node_cpus(0); print(",".join(map(str, sorted(c))) if c else "")')
PIN=""
[ -n "$CPUS" ] && PIN="taskset -c $CPUS"
: > "$OUT/rtt.log"
for round in 1 2; do
  for wgs in 1 2 4 8 16; do
    for door in -; do
      r=$(WSG_LANE_WGS=$wgs timeout -k 10 60 $PIN tools/_build/lane_rtt 32 20000 2>&1 | tail -1) || { echo "fail $wgs $door"; exit 1; }
      echo "wgs=$wgs door=$door $r" >> "$OUT/rtt.log"
    done
  done
done
cat "$OUT/rtt.log"
