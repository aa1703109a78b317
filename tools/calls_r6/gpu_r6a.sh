#!/bin/bash
# Lane re-arm + inline-answer poisoning: the tests, the wrap job against the
# diagnostic build without the poisoning (expected to fail), per-call echo.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6a}
mkdir -p "$OUT"
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_lane.py tests/test_gpu_rx_batch.py tests/test_gpu_session.py tests/test_gpu_cpp_api.py > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
# the same wrap job on the library without the poisoning: expected ok=false
WSG_LIB_PATH=$PWD/cppserver_amd/_build/var/nopoison/libwsg.so WSG_TEST_LANE_TICKET_BASE=$((2**32-300)) WSG_TEST_LANE_STALE_XRES=1 \
  timeout -k 10 90 python -u tests/lane_timeout_job.py wrap > "$OUT/wrap_nopoison.log" 2>&1 || true
tail -c 600 "$OUT/wrap_nopoison.log"; echo
for i in 1 2 3; do
  timeout -k 10 60 tools/_build/bench_echo per_call 1 1 1000 32 2 2>&1 | tail -1 >> "$OUT/per_call.log" || { echo "echo failed"; exit 1; }
done
cat "$OUT/per_call.log"
