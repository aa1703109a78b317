#!/bin/bash
# The differential fuzz with corrupted wires (every third seed), 900 seeds, on the final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5aj}
mkdir -p "$OUT"
export TMPDIR=/tmp
WSG_FUZZ_SEEDS=900 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py -k encode_decode > "$OUT/fuzz_900.log" 2>&1 || { echo "fuzz rc=$?"; tail -40 "$OUT/fuzz_900.log"; exit 1; }
tail -1 "$OUT/fuzz_900.log"
