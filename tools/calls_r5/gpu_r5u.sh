#!/bin/bash
# Tick-sized host batches (100 sessions x 1000 x 38 B = 3.8 MB per pass): read in place ($WSG_HOST_DIRECT_MAX default 4 MB) vs the staged pipeline (=0), per-call GPU pass times and rates
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5u}
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/ab.log"
for round in 1 2; do
  for hd in default 0 1048576; do
    if [ "$hd" = default ]; then unset WSG_HOST_DIRECT_MAX; else export WSG_HOST_DIRECT_MAX=$hd; fi
    r=$(timeout -k 10 60 tools/_build/bench_echo_prof tick 100 1 1000 32 2 2>&1) || { echo "fail prof $hd"; exit 1; }
    echo "host_direct_max=$hd tick 100 1: $(echo "$r" | python3 -c '
import sys,json
lines=sys.stdin.read().splitlines()
p=json.loads([l for l in lines if l.startswith("ECHO_PROF")][0][10:])
d=json.loads(lines[-1])
print(d["msg_per_s"], d["payload_ok"], "dec_us", p["gpu_decode_host"]["us_per_call"], "enc_us", p["gpu_encode_host"]["us_per_call"])')" >> "$OUT/ab.log"
    r=$(timeout -k 10 60 tools/_build/bench_echo_tcp gpu_tick 100 4 1000 32 2 2>&1 | tail -1) || { echo "fail tcp $hd"; exit 1; }
    echo "host_direct_max=$hd tcp gpu_tick 100 4: $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["msg_per_s"], d["payload_ok"], d["lane_requests"], d["reads"])')" >> "$OUT/ab.log"
  done
done
unset WSG_HOST_DIRECT_MAX
cat "$OUT/ab.log"
