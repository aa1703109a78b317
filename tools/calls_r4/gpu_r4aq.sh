#!/bin/bash
# Final tree (lane cap from GPU_MAX_HW_QUEUES included): the full GPU suite, then smoke()
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4aq}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== suite $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/suite.log" 2>&1
rc=$?
tail -3 "$OUT/suite.log"
[ $rc -ne 0 ] && exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
rc=$?
tail -2 "$OUT/smoke.log"
exit $rc
