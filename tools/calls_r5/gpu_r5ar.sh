#!/bin/bash
# Final tree: bench.py --gpus 2 (two ranks on the one GPU: the N > 1 path the driver's scaling run takes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5ar}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_BENCH_SHARE_DEVICES=1 timeout -k 10 900 python bench.py --gpus 2 > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" || { echo "bench n2 rc=$?"; tail -30 "$OUT/bench_n2.err"; exit 1; }
python3 - "$OUT/bench_n2.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d.get(k) for k in ("metric", "value", "n_gpus", "scaling", "ms_per_step", "failed_checks")})
print({k: v for k, v in d.get("c5_job", {}).items() if k in ("encode_ms", "gather_ms", "root_check", "GBps_into_root", "path")})
PY
