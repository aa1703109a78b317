#!/bin/bash
# Bounds fuzz: exact-size outputs with a sentinel behind them, every entry point
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6o}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_FUZZ_SEEDS=1500 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k nothing_written_past > "$OUT/bounds_fuzz.log" 2>&1 || { echo "bounds fuzz rc=$?"; grep -E "FAILED|Error|assert" "$OUT/bounds_fuzz.log" | head -30; tail -5 "$OUT/bounds_fuzz.log"; exit 1; }
tail -n 1 "$OUT/bounds_fuzz.log"
