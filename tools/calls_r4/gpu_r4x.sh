#!/bin/bash
# Round-4 bench line: the driver's command (python bench.py --steps 20 --warmup 5)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/art_r4
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== bench $(date +%T)"
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > "$OUT/bench.out" 2> "$OUT/bench.err"
rc=$?
echo "rc=$rc $(date +%T)"
tail -c 3000 "$OUT/bench.out"
exit $rc
