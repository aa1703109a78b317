#!/bin/bash
# Per-call echo latency vs where the host thread runs: the box's CPU set, NUMA nodes and the GPU's node, then bench_echo per_call pinned to CPUs of each node
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5aa}
mkdir -p "$OUT"
export TMPDIR=/tmp
{
  echo "allowed: $(grep Cpus_allowed_list /proc/self/status)"
  for n in /sys/devices/system/node/node*; do echo "$(basename $n): $(cat $n/cpulist)"; done
  for d in /sys/class/drm/card*/device; do [ -f $d/numa_node ] && echo "$d numa_node=$(cat $d/numa_node)"; done
  echo "HIP_VISIBLE_DEVICES=${HIP_VISIBLE_DEVICES:-} ROCR_VISIBLE_DEVICES=${ROCR_VISIBLE_DEVICES:-}"
} > "$OUT/topo.log" 2>&1
cat "$OUT/topo.log"
allowed=$(python3 -c 'import os; print(" ".join(map(str, sorted(os.sched_getaffinity(0)))))')
: > "$OUT/pin.log"
for n in /sys/devices/system/node/node*; do
  node=$(basename $n)
  cpu=$(python3 - "$n/cpulist" "$allowed" <<'PY'
import sys
spec=open(sys.argv[1]).read().strip()
allowed=set(map(int, sys.argv[2].split()))
cpus=[]
for part in spec.split(','):
    if '-' in part:
        a,b=map(int,part.split('-')); cpus+=range(a,b+1)
    elif part: cpus.append(int(part))
ok=[c for c in cpus if c in allowed]
print(ok[len(ok)//2] if ok else "")
PY
)
  [ -z "$cpu" ] && { echo "$node: no allowed cpu" >> "$OUT/pin.log"; continue; }
  for round in 1 2; do
    r=$(timeout -k 10 60 taskset -c $cpu tools/_build/bench_echo per_call 1 1 1000 32 2 2>&1 | tail -1) || { echo "fail $node"; exit 1; }
    echo "$node cpu $cpu per_call $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["msg_per_s"], d["payload_ok"])')" >> "$OUT/pin.log"
  done
done
cat "$OUT/pin.log"
