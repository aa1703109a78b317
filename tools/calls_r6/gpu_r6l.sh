#!/bin/bash
# Debug: bytes a many-message fan-out writes outside its frames (fuzz seed 123), product vs round 5's shape
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6l}
mkdir -p "$OUT"
timeout -k 10 60 python -u tools/fan_gap_dbg.py 123 > "$OUT/product.log" 2>&1 || { echo "rc=$?"; cat "$OUT/product.log"; exit 1; }
WSG_LIB_PATH=$PWD/cppserver_amd/_build/var/old/libwsg.so timeout -k 10 60 python -u tools/fan_gap_dbg.py 123 > "$OUT/old.log" 2>&1 || { echo "rc=$?"; cat "$OUT/old.log"; exit 1; }
tail -n 25 "$OUT/product.log"; echo ==== old; tail -n 8 "$OUT/old.log"
