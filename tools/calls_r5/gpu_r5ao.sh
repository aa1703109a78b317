#!/bin/bash
# Final tree (lane on the near XCDs): full GPU suite, smoke, the driver's bench command; then the idle-poller probe (gpu_r5an.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5ao}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu suite rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C2", d["value"], d["roofline"]["frac"], "C3", d["c3"]["roofline"]["halves"][0]["frac"], d["c3"]["roofline"]["halves"][1]["frac"],
      "C4", d["c4"]["roofline"]["frac"], "C5", d["c5"]["roofline"]["frac"], "host_legs", d.get("host_legs_cpus", {}).get("numa_node"))
e = d["echo_c1"]
print({k: e[k]["msg_per_s"] for k in ("per_read_1c", "per_read_100c_4t", "tick_100c_1t", "per_call_1c")},
      "tcp100", e["tcp_loopback"]["gpu_100c_4t"]["msg_per_s"], "ref", e["tcp_loopback"]["cpu_ref_100c_4t"]["msg_per_s"])
print("failed", d["failed_checks"])
PY
TAG=r5an bash tools/calls_r5/gpu_r5an.sh | tail -10
