#!/bin/bash
# Lanes per process: none, all, capped (WSG_LANE_CAP) over the echo modes (in-memory and TCP)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4ae}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc $(python -c "import json; print(json.loads(open('$OUT/$name.log').read().strip().splitlines()[-1])['msg_per_s'])" 2>/dev/null)"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
    return 0
}
for v in "WSG_LANE_MAX=0" "WSG_LANE_CAP=1000" "WSG_LANE_CAP=1" "WSG_LANE_CAP=2" "WSG_LANE_CAP=4"; do
  t=${v//=/_}
  step mem_1c_$t 60 env $v tools/_build/bench_echo per_read 1 1 1000 32 2
  step mem_100c_$t 60 env $v tools/_build/bench_echo per_read 100 4 1000 32 2
  step mem_tick_$t 60 env $v tools/_build/bench_echo tick 100 1 1000 32 2
  step tcp_1c_$t 60 env $v tools/_build/bench_echo_tcp gpu 1 1 1000 32 2
  step tcp_100c_$t 60 env $v tools/_build/bench_echo_tcp gpu 100 4 1000 32 2
  step tcp_tick_$t 60 env $v tools/_build/bench_echo_tcp gpu_tick 100 4 1000 32 2
done
step ref_mem_1c 60 tools/_build/bench_echo_ref -c 1 -t 1 -m 1000 -s 32 -z 2
step ref_mem_100c 60 tools/_build/bench_echo_ref -c 100 -t 4 -m 1000 -s 32 -z 2
step ref_tcp_1c 60 tools/_build/bench_echo_tcp cpu_ref 1 1 1000 32 2
step ref_tcp_100c 60 tools/_build/bench_echo_tcp cpu_ref 100 4 1000 32 2
echo "== done"
