#!/bin/bash
# Does a second poller slow the first?  tools/xcd_probe.hip: block 0 serves the host ping-pong while 0-15 other blocks poll page-locked words of their own
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5an}
mkdir -p "$OUT"
export TMPDIR=/tmp
CPUS=$(timeout -k 10 120 python3 -c 'import sys; sys.path.insert(0, "."); import bench; n, c = bench.gpu_node_cpus(0); print(",".join(map(str, sorted(c))) if c else "")')
PIN=""
[ -n "$CPUS" ] && PIN="taskset -c $CPUS"
: > "$OUT/noise.log"
for round in 1 2; do
  for noise in 0 1 3 7 15; do
    timeout -k 10 60 $PIN tools/_build/xcd_probe 1 20000 $noise >> "$OUT/noise.log" 2>&1 || { echo "probe rc=$?"; cat "$OUT/noise.log"; exit 1; }
  done
done
cat "$OUT/noise.log"
