#!/bin/bash
# The TCP echo, 100 clients on 4+4 threads, ten runs each of the drop-in
# classes and the reference algorithm, alternating, with the lane's counters
# (one 29.8 M outlier in round 5)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6x}
mkdir -p "$OUT"
: > "$OUT/tcp_repeat.log"
for i in $(seq 1 10); do
  for m in gpu cpu_ref; do
    timeout -k 10 60 tools/_build/bench_echo_tcp $m 100 4 1000 32 3 2>&1 | tail -n 1 >> "$OUT/tcp_repeat.log" || { echo "rc=$? $m"; exit 1; }
  done
done
python3 -c '
import json
rows=[json.loads(l) for l in open("'"$OUT"'/tcp_repeat.log") if l.startswith("{")]
for c in ("gpu","cpu_ref"):
    v=sorted(r["msg_per_s"] for r in rows if r["codec"]==c)
    print(c, [round(x/1e6,1) for x in v], "give_ups", sorted(set(r.get("lane_give_ups") for r in rows if r["codec"]==c)))'
