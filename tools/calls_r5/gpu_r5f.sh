#!/bin/bash
# Lane tests (incl. timeout and constant hand-over in their own processes), the fan-out parity tests, the C++ API tests, then the bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lane.py tests/test_gpu_cpp_api.py "tests/test_gpu_parity.py" -k "lane or fanout or cpp or echo or concurrent" > "$OUT/tests.log" 2>&1 || { echo "tests rc=$?"; tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e=d.get("echo_c1",{})
print("value",d["value"],"frac",d["roofline"]["frac"],"traffic",d["roofline"]["traffic"],"failed",d["failed_checks"])
print("per_call_1c",e.get("per_call_1c",{}).get("msg_per_s"),"per_read_1c",e.get("per_read_1c",{}).get("msg_per_s"))
t=e.get("tcp_loopback",{})
print({k:v.get("msg_per_s") for k,v in t.items() if isinstance(v,dict)})
c4=d.get("c4",{})
print("c4",c4.get("roofline",{}).get("frac"),"tick",c4.get("multicast_tick_16",{}).get("us_per_call"),c4.get("multicast_tick_16",{}).get("bare_write_stream",{}).get("fanout_vs_bare"))
PY
