#!/bin/bash
# Full GPU suite and the bench line after pruning the compile-time A/B variants (regression check)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu suite rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
run() { local name=$1; shift; timeout -k 10 60 "$@" > "$OUT/$name.log" 2>&1 || { echo "$name rc=$?"; tail -5 "$OUT/$name.log"; exit 1; }; echo "$name $(tail -1 "$OUT/$name.log" | cut -c1-220)"; }
run mem_per_call tools/_build/bench_echo per_call 1 1 1000 32 3
run mem_per_read tools/_build/bench_echo per_read 1 1 1000 32 3
run tcp_gpu_100c tools/_build/bench_echo_tcp gpu 100 4 1000 32 3
run tcp_ref_100c tools/_build/bench_echo_tcp cpu_ref 100 4 1000 32 3
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e=d.get("echo_c1",{})
print("value",d["value"],"frac",d["roofline"]["frac"],"failed",d["failed_checks"])
print("per_call_1c",e.get("per_call_1c",{}).get("msg_per_s"),"per_read_1c",e.get("per_read_1c",{}).get("msg_per_s"))
t=e.get("tcp_loopback",{})
print({k:v.get("msg_per_s") for k,v in t.items() if isinstance(v,dict)})
print("c4",d.get("c4",{}).get("roofline",{}).get("frac"))
PY
