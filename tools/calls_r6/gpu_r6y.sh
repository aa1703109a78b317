#!/bin/bash
# Session batching fuzz on the final tree: 600 seeds each of the batched receive and send fuzz
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6y}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_FUZZ_SEEDS=600 timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx_batch.py tests/test_gpu_tx_batch.py -k fuzz > "$OUT/rxtx_fuzz_600.log" 2>&1 || { echo "rxtx fuzz rc=$?"; grep -E "FAILED|Error" "$OUT/rxtx_fuzz_600.log" | head; tail -5 "$OUT/rxtx_fuzz_600.log"; exit 1; }
tail -n 1 "$OUT/rxtx_fuzz_600.log"
