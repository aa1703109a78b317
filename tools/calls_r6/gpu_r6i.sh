#!/bin/bash
# Full GPU suite, smoke, the driver's bench command, and the N=2 rehearsal
# (ranks sharing the one GPU) with the RCCL banners counted.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu suite rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -n 1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
python3 -c '
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "frac", d["roofline"]["frac"], "failed", d["failed_checks"])
fm=d.get("c4",{}).get("fanout_many") or d.get("c4",{})
print("c4", json.dumps(d.get("c4",{}))[:1500])
print("echo", json.dumps(d.get("echo_c1",{}))[:1500])
' "$OUT/bench.json"
NCCL_DEBUG=VERSION WSG_BENCH_SHARE_DEVICES=1 timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" || { echo "bench n2 rc=$?"; tail -30 "$OUT/bench_n2.err"; exit 1; }
grep -c "RCCL version" "$OUT/bench_n2.json" "$OUT/bench_n2.err" || true
grep -h "RCCL version" "$OUT/bench_n2.json" "$OUT/bench_n2.err" | sort | uniq -c || true
tail -c 1500 "$OUT/bench_n2.json"
