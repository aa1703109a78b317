#!/bin/bash
# The widest fuzz campaign of the round: 5000 seeds of every differential fuzz
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6w}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_FUZZ_SEEDS=5000 timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py > "$OUT/fuzz_5000.log" 2>&1 || { echo "fuzz rc=$?"; grep -E "FAILED|Error" "$OUT/fuzz_5000.log" | head -20; tail -5 "$OUT/fuzz_5000.log"; exit 1; }
tail -n 1 "$OUT/fuzz_5000.log"
