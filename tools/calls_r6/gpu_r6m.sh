#!/bin/bash
# The period kernel's partial last row: the regression test against the
# round-5-shape build (expected to fail) and the product, the fan-out parity
# tests, then the 2000-seed fuzz campaign and the rx/tx session fuzz.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6m}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_LIB_PATH=$PWD/cppserver_amd/_build/var/old/libwsg.so timeout -k 10 200 python -u -m pytest -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py -k last_chunk_partial > "$OUT/old_build.log" 2>&1
echo "old build (round-5 kernel): $(tail -n 1 "$OUT/old_build.log")"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k fanout > "$OUT/parity_fanout.log" 2>&1 || { echo "parity rc=$?"; tail -30 "$OUT/parity_fanout.log"; exit 1; }
tail -n 1 "$OUT/parity_fanout.log"
WSG_FUZZ_SEEDS=2000 timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py > "$OUT/fuzz_2000.log" 2>&1 || { echo "fuzz rc=$?"; tail -30 "$OUT/fuzz_2000.log"; exit 1; }
tail -n 1 "$OUT/fuzz_2000.log"
WSG_FUZZ_SEEDS=200 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rx_batch.py tests/test_gpu_tx_batch.py -k fuzz > "$OUT/rxtx_fuzz_200.log" 2>&1 || { echo "rxtx fuzz rc=$?"; tail -30 "$OUT/rxtx_fuzz_200.log"; exit 1; }
tail -n 1 "$OUT/rxtx_fuzz_200.log"
