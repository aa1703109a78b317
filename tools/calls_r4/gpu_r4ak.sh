#!/bin/bash
# Fan-out grid path: parity tests, then 16 x C4 in one call vs the period path and the bare fill
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4ak}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fanout" -x -q --timeout 300 --timeout-method thread > "$OUT/fan_tests.log" 2>&1
rc=$?
tail -3 "$OUT/fan_tests.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/fan_many_ab.py "" "WSG_FAN_GRID=0" > "$OUT/fan_many_ab.log" 2>&1 || { tail -20 "$OUT/fan_many_ab.log"; exit 1; }
tail -1 "$OUT/fan_many_ab.log"
