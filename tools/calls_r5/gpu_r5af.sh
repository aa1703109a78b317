#!/bin/bash
# One lane task's round trip on the per-call path (tools/lane_rtt.cpp): mailboxes in device vs host memory, 32 B inline and 1 KiB staged XORs, host thread on the GPU's NUMA node; and the BAR probe again
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5af}
mkdir -p "$OUT"
export TMPDIR=/tmp
CPUS=$(timeout -k 10 120 python3 -c 'import sys; sys.path.insert(0, "."); import bench; n, c = bench.gpu_node_cpus(0); print(",".join(map(str, sorted(c))) if c else "")')
PIN=""
[ -n "$CPUS" ] && PIN="taskset -c $CPUS"
: > "$OUT/rtt.log"
for round in 1 2; do
  for door in 1 0; do
    for size in 32 1024; do
      r=$(WSG_LANE_DOOR=$door timeout -k 10 60 $PIN tools/_build/lane_rtt $size 20000 2>&1 | tail -1) || { echo "fail $door $size"; exit 1; }
      echo "door=$door $r" >> "$OUT/rtt.log"
    done
  done
done
timeout -k 10 60 $PIN tools/_build/bar_probe 20000 >> "$OUT/rtt.log" 2>&1 || { echo "probe failed"; exit 1; }
cat "$OUT/rtt.log"
