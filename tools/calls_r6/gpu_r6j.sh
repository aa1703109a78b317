#!/bin/bash
# Lane tests (incl. the churn case: given up and re-armed under eight
# threads), then the many-message fan-out against round 5's launch shape
# ("old": 4-workgroup cap, 6 waves per CU) at 4, 8 and 32 messages per tick.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lane.py > "$OUT/lane.log" 2>&1 || { echo "lane tests rc=$?"; tail -30 "$OUT/lane.log"; exit 1; }
tail -n 2 "$OUT/lane.log"
: > "$OUT/fan_m.log"
for m in 4 8 32; do
  for round in 1 2; do
    for v in base old; do
      if [ "$v" = base ]; then lib=cppserver_amd/_build/libwsg.so; else lib=cppserver_amd/_build/var/$v/libwsg.so; fi
      M=$m ROUNDS=3 timeout -k 10 120 python tools/fan_ab.py $v=$lib >> "$OUT/fan_m.log" 2>&1 || { echo "ab $v m=$m rc=$?"; tail -20 "$OUT/fan_m.log"; exit 1; }
    done
  done
done
grep '^{' "$OUT/fan_m.log" | python3 -c '
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(r["variant"], r["m"], r["tick_us"], r["fill_us"], r["tick_vs_fill"], not r["parity_bad"] and r["c4_ok"])'
