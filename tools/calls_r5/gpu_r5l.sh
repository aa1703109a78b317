#!/bin/bash
# Pageable host batches with the parallel staging copies: the host-path parity tests, then the bench line (pcie_inclusive_GiBps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_host_multi.py tests/test_gpu_tx_batch.py tests/test_gpu_rx_batch.py > "$OUT/host_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/host_tests.log"; exit 1; }
tail -1 "$OUT/host_tests.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value",d["value"],"frac",d["roofline"]["frac"],"failed",d["failed_checks"])
print("pcie",d.get("pcie_inclusive_GiBps"))
print("session_batch",{k:(v.get("batched_GiBps"),v.get("per_call_GiBps")) for k,v in d.get("session_batch",{}).items() if isinstance(v,dict)})
PY
