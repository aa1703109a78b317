#!/bin/bash
# Final-tree evidence: 2000-seed differential fuzz (decode/encode/fan-out, and
# the many-message fan-out at 1000 seeds), 200-seed rx/tx session fuzz, and
# the bench line with the C4 per-launch events.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6k}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_FUZZ_SEEDS=2000 timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py > "$OUT/fuzz_2000.log" 2>&1 || { echo "fuzz rc=$?"; tail -30 "$OUT/fuzz_2000.log"; exit 1; }
tail -n 1 "$OUT/fuzz_2000.log"
WSG_FUZZ_SEEDS=200 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx_batch.py tests/test_gpu_tx_batch.py -k fuzz > "$OUT/rxtx_fuzz_200.log" 2>&1 || { echo "rxtx fuzz rc=$?"; tail -30 "$OUT/rxtx_fuzz_200.log"; exit 1; }
tail -n 1 "$OUT/rxtx_fuzz_200.log"
