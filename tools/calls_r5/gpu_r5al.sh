#!/bin/bash
# Host-memory ping-pong round trip by the block (and XCC) the poller runs on (tools/xcd_probe.hip), host thread on the GPU's NUMA node
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5al}
mkdir -p "$OUT"
export TMPDIR=/tmp
CPUS=$(timeout -k 10 120 python3 -c 'import sys; sys.path.insert(0, "."); import bench; n, c = bench.gpu_node_cpus(0); print(",".join(map(str, sorted(c))) if c else "")')
PIN=""
[ -n "$CPUS" ] && PIN="taskset -c $CPUS"
timeout -k 10 120 $PIN tools/_build/xcd_probe 16 20000 > "$OUT/xcd.log" 2>&1 || { echo "probe rc=$?"; cat "$OUT/xcd.log"; exit 1; }
cat "$OUT/xcd.log"
