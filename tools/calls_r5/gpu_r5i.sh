#!/bin/bash
# Differential fuzz on the round's final kernels and lane: 2000 seeds of the batch codec (device and host-staged,
# incl. fan-outs), 200 of the batched receive and of the batched send, against the oracle
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5i}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_FUZZ_SEEDS=2000 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py > "$OUT/fuzz_2000.log" 2>&1 || { echo "fuzz rc=$?"; tail -30 "$OUT/fuzz_2000.log"; exit 1; }
tail -1 "$OUT/fuzz_2000.log"
WSG_FUZZ_SEEDS=200 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx_batch.py tests/test_gpu_tx_batch.py -k fuzz > "$OUT/rxtx_fuzz_200.log" 2>&1 || { echo "rxtx fuzz rc=$?"; tail -30 "$OUT/rxtx_fuzz_200.log"; exit 1; }
tail -1 "$OUT/rxtx_fuzz_200.log"
