#!/bin/bash
# Large in-place decodes read the error latch back instead of scanning the records: lane / rx-batch / session tests, the tick echo's per-call times, the 32-byte session batches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5x}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lane.py tests/test_gpu_rx_batch.py tests/test_gpu_session.py > "$OUT/tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
: > "$OUT/echo.log"
for round in 1 2; do
  r=$(timeout -k 10 60 tools/_build/bench_echo_prof tick 100 1 1000 32 2 2>&1) || { echo "fail prof"; exit 1; }
  echo "tick 100 1: $(echo "$r" | python3 -c '
import sys,json
lines=sys.stdin.read().splitlines()
p=json.loads([l for l in lines if l.startswith("ECHO_PROF")][0][10:])
d=json.loads(lines[-1])
print(d["msg_per_s"], d["payload_ok"], "dec_us", p["gpu_decode_host"]["us_per_call"], "enc_us", p["gpu_encode_host"]["us_per_call"])')" >> "$OUT/echo.log"
  r=$(timeout -k 10 120 tools/_build/bench_batch rx 256 64 32 0 3 2>&1 | tail -1) || { echo "fail batch"; exit 1; }
  echo "bench_batch rx 32B $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["batched_frames_per_s"], d["delivered_ok"])')" >> "$OUT/echo.log"
done
cat "$OUT/echo.log"
