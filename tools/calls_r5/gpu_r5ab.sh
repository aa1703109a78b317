#!/bin/bash
# The driver's bench command with the host legs bound to the GPU's NUMA node
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C2", d["value"], d["roofline"]["frac"], "host_legs", d.get("host_legs_cpus"))
e = d["echo_c1"]
for k in ("per_read_1c", "per_read_100c_4t", "tick_100c_1t", "per_call_1c", "wss_per_read_1c"):
    print(k, e[k]["msg_per_s"])
print("cpu_ref", e["cpu_reference"]["1c_1t"]["msg_per_s"], e["cpu_reference"]["100c_4t"]["msg_per_s"])
for k, v in e["tcp_loopback"].items():
    if isinstance(v, dict) and "msg_per_s" in v:
        print(k, v["msg_per_s"], v.get("runs_msg_per_s"))
print("failed", d["failed_checks"])
PY
