#!/bin/bash
# Inline per-call answers (self-tagged units, no fence): lane + session + C++ API tests, then the per-call and per-read echo legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lane.py tests/test_gpu_session.py tests/test_gpu_cpp_api.py > "$OUT/tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for round in 1 2; do
  for leg in "bench_echo per_call 1 1" "bench_echo per_read 1 1" "bench_echo_tcp gpu 100 4"; do
    set -- $leg
    exe=$1; shift
    r=$(timeout -k 10 60 tools/_build/$exe "$@" 1000 32 2 2>&1 | tail -1) || { echo "fail $leg"; exit 1; }
    echo "$leg $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["msg_per_s"], d["payload_ok"])')" | tee -a "$OUT/echo.log"
  done
done
