#!/bin/bash
# Lane mailboxes in device memory (the door, stored into over the BAR) vs page-locked host memory ($WSG_LANE_DOOR=0): lane / session / C++ API tests, then the echo legs interleaved, host threads on the GPU's NUMA node
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5ad}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lane.py tests/test_gpu_session.py tests/test_gpu_cpp_api.py > "$OUT/tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
CPUS=$(timeout -k 10 120 python3 -c 'import sys; sys.path.insert(0, "."); import bench; n, c = bench.gpu_node_cpus(0); print(",".join(map(str, sorted(c))) if c else "")')
echo "gpu node cpus: ${CPUS:0:40}..." > "$OUT/ab.log"
PIN=""
[ -n "$CPUS" ] && PIN="taskset -c $CPUS"
for round in 1 2; do
  for door in 1 0; do
    export WSG_LANE_DOOR=$door
    for leg in "bench_echo per_call 1 1" "bench_echo per_read 1 1" "bench_echo per_read 100 4" "bench_echo_tcp gpu 100 4"; do
      set -- $leg
      exe=$1; shift
      r=$(timeout -k 10 60 $PIN tools/_build/$exe "$@" 1000 32 2 2>&1 | tail -1) || { echo "fail $door $leg"; exit 1; }
      echo "door=$door $leg $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["msg_per_s"], d["payload_ok"])')" >> "$OUT/ab.log"
    done
  done
done
unset WSG_LANE_DOOR
cat "$OUT/ab.log"
