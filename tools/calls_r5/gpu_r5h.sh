#!/bin/bash
# The full GPU suite and smoke on the current tree, then the N=2 command rehearsed with both ranks on the one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5h}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu suite rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
WSG_BENCH_SHARE_DEVICES=1 timeout -k 10 500 python bench.py --gpus 2 --steps 20 --warmup 5 > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" || { echo "n2 rc=$?"; tail -30 "$OUT/bench_n2.err"; exit 1; }
python - "$OUT/bench_n2.json" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1])
print("n_gpus",d["n_gpus"],"value",d["value"],"failed",d["failed_checks"])
print({k: (v if not isinstance(v, dict) else {kk: vv for kk, vv in v.items() if not isinstance(vv, (dict, list))}) for k, v in d.items() if k.startswith("c5")})
PY
