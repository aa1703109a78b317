#!/bin/bash
# One GPU call: pytest -m gpu + smoke, then the round's measurement artifacts
# (tools/round_artifacts.sh).  usage: gpurun -- bash tools/gpu_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/full
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/full/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/full/smoke.log
ROUND=${ROUND:?set ROUND} bash tools/round_artifacts.sh
