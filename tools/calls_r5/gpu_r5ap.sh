#!/bin/bash
# Why do idle pollers speed the ping-pong up?  tools/xcd_probe.hip: noise pollers reading the server's word too vs only their own; the server block with 1-16 staggered waves
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5ap}
mkdir -p "$OUT"
export TMPDIR=/tmp
CPUS=$(timeout -k 10 120 python3 -c 'import sys; sys.path.insert(0, "."); import bench; n, c = bench.gpu_node_cpus(0); print(",".join(map(str, sorted(c))) if c else "")')
PIN=""
[ -n "$CPUS" ] && PIN="taskset -c $CPUS"
: > "$OUT/probe.log"
for round in 1 2; do
  for args in "0 0 1" "15 0 1" "15 1 1" "31 1 1" "0 0 2" "0 0 4" "0 0 8" "0 0 16"; do
    timeout -k 10 60 $PIN tools/_build/xcd_probe 1 20000 $args >> "$OUT/probe.log" 2>&1 || { echo "probe rc=$? ($args)"; tail -3 "$OUT/probe.log"; exit 1; }
  done
done
cat "$OUT/probe.log"
