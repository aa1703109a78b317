#!/bin/bash
# Pipelined lane polling (two reads of the slot in flight, 8-byte self-tagged task units) vs the committed lane (var/pre_pipe): the inline-XOR round trip first (no task pointer is dereferenced), then the lane / session / C++ API / rx-batch tests, then echo legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5as}
mkdir -p "$OUT"
export TMPDIR=/tmp
CPUS=$(timeout -k 10 120 python3 -c 'import sys; sys.path.insert(0, "."); import bench; n, c = bench.gpu_node_cpus(0); print(",".join(map(str, sorted(c))) if c else "")')
PIN=""
[ -n "$CPUS" ] && PIN="taskset -c $CPUS"
r=$(timeout -k 10 60 $PIN tools/_build/lane_rtt 32 20000 2>&1 | tail -1) || { echo "rtt failed: $r"; exit 1; }
echo "first rtt: $r"
echo "$r" | grep -q '"bytes_ok": true' || { echo "inline XOR wrong: stop"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lane.py tests/test_gpu_session.py tests/test_gpu_cpp_api.py tests/test_gpu_rx_batch.py > "$OUT/tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
: > "$OUT/ab.log"
for round in 1 2; do
  for v in product pre_pipe; do
    if [ "$v" = product ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=$PWD/cppserver_amd/_build/var/pre_pipe; fi
    r=$(timeout -k 10 60 $PIN tools/_build/lane_rtt 32 20000 2>&1 | tail -1) || { echo "fail rtt $v"; exit 1; }
    echo "$v lane_rtt $r" >> "$OUT/ab.log"
    for leg in "bench_echo per_call 1 1" "bench_echo per_read 1 1" "bench_echo per_read 100 4" "bench_echo_tcp gpu 100 4"; do
      set -- $leg
      exe=$1; shift
      r=$(timeout -k 10 60 $PIN tools/_build/$exe "$@" 1000 32 2 2>&1 | tail -1) || { echo "fail $v $leg"; exit 1; }
      echo "$v $leg $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["msg_per_s"], d["payload_ok"])')" >> "$OUT/ab.log"
    done
  done
done
unset LD_LIBRARY_PATH
cat "$OUT/ab.log"
