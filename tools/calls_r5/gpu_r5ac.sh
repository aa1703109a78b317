#!/bin/bash
# Doorbell in device memory written over the BAR vs in page-locked host memory (tools/bar_probe.hip): host access to fine-grained / uncached device memory and ping-pong round trips
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5ac}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 tools/_build/bar_probe 20000 > "$OUT/bar_probe.log" 2>&1
echo "rc=$?" >> "$OUT/bar_probe.log"
cat "$OUT/bar_probe.log"
