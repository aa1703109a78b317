#!/bin/bash
# Fan-out A/B (tools/fan_ab.py): period kernel with its workgroups per CU capped (LDS reserve), key registers 2 vs 4
# One process per variant (each library's initial-exec TLS), variants interleaved over rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5e}
mkdir -p "$OUT"
V=cppserver_amd/_build/var
: > "$OUT/fan_run_ab.log"
for round in 1 2 3; do
  for v in ${VARIANTS:-period cap3kv4 cap4kv4 cap5kv4 cap6kv4 cap8}; do
    ROUNDS=3 timeout -k 10 120 python tools/fan_ab.py $v=$V/$v/libwsg.so >> "$OUT/fan_run_ab.log" 2>&1 || { echo "ab $v rc=$?"; tail -20 "$OUT/fan_run_ab.log"; exit 1; }
  done
done
cat "$OUT/fan_run_ab.log"
