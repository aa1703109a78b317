#!/bin/bash
# Per-call echo (batching off): product library vs the library before the byte-grouped lane requests (var/pre_groups, via LD_LIBRARY_PATH), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5z}
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/ab.log"
for round in 1 2 3; do
  for v in product pre_groups; do
    if [ "$v" = product ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=$PWD/cppserver_amd/_build/var/pre_groups; fi
    for leg in "per_call 1 1" "per_read 1 1"; do
      r=$(timeout -k 10 60 tools/_build/bench_echo $leg 1000 32 2 2>&1 | tail -1) || { echo "fail $v $leg"; exit 1; }
      echo "$v $leg $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["msg_per_s"], d["payload_ok"])')" >> "$OUT/ab.log"
    done
  done
done
unset LD_LIBRARY_PATH
cat "$OUT/ab.log"
