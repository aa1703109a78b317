#!/bin/bash
# BAR probe with the host's task-store times, plain and with the lane's store fences, host thread on the GPU's NUMA node
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5ag}
mkdir -p "$OUT"
export TMPDIR=/tmp
CPUS=$(timeout -k 10 120 python3 -c 'import sys; sys.path.insert(0, "."); import bench; n, c = bench.gpu_node_cpus(0); print(",".join(map(str, sorted(c))) if c else "")')
PIN=""
[ -n "$CPUS" ] && PIN="taskset -c $CPUS"
timeout -k 10 90 $PIN tools/_build/bar_probe 20000 > "$OUT/probe.log" 2>&1 || { echo "probe failed"; cat "$OUT/probe.log"; exit 1; }
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); [print(k, v) for k, v in d.items() if "attr" not in k]' "$OUT/probe.log"
