#!/bin/bash
# Drain's private delivery on the thread's own codec: C++ API tests (incl.
# the keyed cross-thread drain), rx/tx batch and session tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6n}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cpp_api.py tests/test_gpu_rx_batch.py tests/test_gpu_tx_batch.py tests/test_gpu_session.py > "$OUT/tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/tests.log"; exit 1; }
tail -n 1 "$OUT/tests.log"
timeout -k 10 120 tests/cpp/_build/test_ws_api > "$OUT/test_ws_api.log" 2>&1 || { echo "ws_api rc=$?"; tail -20 "$OUT/test_ws_api.log"; exit 1; }
tail -n 1 "$OUT/test_ws_api.log"
