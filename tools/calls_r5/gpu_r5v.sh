#!/bin/bash
# After the byte-grouped lane requests: full GPU suite, smoke, the driver's bench command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5v}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu suite rc=$?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
