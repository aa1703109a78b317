#!/bin/bash
# The driver's round-end commands on the final tree: the GPU suite as the
# driver runs it, smoke, and the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6v}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu suite rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -n 1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
grep '^{' "$OUT/bench.json" | tail -n 1 | python3 -c '
import json,sys
d=json.loads(sys.stdin.read())
t=d["c4"]["multicast_tick_16"]
print("C2", d["value"], d["roofline"]["frac"], "C3", [h["frac"] for h in d["c3"]["roofline"]["halves"]], "C4", d["c4"]["roofline"]["frac"], "tick", t["us_per_call"], t["bare_write_stream"]["fanout_vs_bare"], "C5", d["c5"]["roofline"]["frac"], "failed", d["failed_checks"])'
