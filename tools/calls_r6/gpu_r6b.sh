#!/bin/bash
# Fan-out A/B (tools/fan_ab.py): the many-message launch's waves per CU per
# message, its workgroups-per-CU cap, and the stores' cache policy; one
# process per variant, variants interleaved over rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6b}
mkdir -p "$OUT"
V=cppserver_amd/_build/var
: > "$OUT/fan_ab.log"
for round in 1 2 3; do
  for v in ${VARIANTS:-base wpc12 wpc24 wpc48 wpc160 cap2w24 cap8w24 cap0w24 aux17}; do
    if [ "$v" = base ]; then lib=cppserver_amd/_build/libwsg.so; else lib=$V/$v/libwsg.so; fi
    ROUNDS=3 timeout -k 10 120 python tools/fan_ab.py $v=$lib >> "$OUT/fan_ab.log" 2>&1 || { echo "ab $v rc=$?"; tail -20 "$OUT/fan_ab.log"; exit 1; }
  done
done
grep '^{' "$OUT/fan_ab.log" | python3 -c '
import sys, json, collections
d = collections.defaultdict(list)
for l in sys.stdin:
    r = json.loads(l); d[r["variant"]].append((r["tick_vs_fill"], r["tick_us"], r["fill_us"], r["c4_us"], not r["parity_bad"] and r["c4_ok"]))
for k, v in d.items(): print(k, v)'
