#!/bin/bash
# Round-4 PMC passes (FETCH_SIZE / WRITE_SIZE per config + membench calibration)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROUND=r4 PMC=1 BENCH=0 bash tools/round_artifacts.sh
