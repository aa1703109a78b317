#!/bin/bash
# N=4 rehearsal of the driver's scaling command with the four ranks sharing the one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6s}
mkdir -p "$OUT"
export TMPDIR=/tmp
NCCL_DEBUG=VERSION WSG_BENCH_SHARE_DEVICES=1 timeout -k 10 900 python bench.py --gpus 4 --steps 20 --warmup 5 > "$OUT/bench_n4.json" 2> "$OUT/bench_n4.err" || { echo "bench n4 rc=$?"; tail -30 "$OUT/bench_n4.err"; exit 1; }
grep -h "RCCL version" "$OUT/bench_n4.json" "$OUT/bench_n4.err" | sort | uniq -c || true
grep '^{' "$OUT/bench_n4.json" | tail -n 1 | python3 -c '
import json,sys
d=json.loads(sys.stdin.read())
print("n_gpus", d["n_gpus"], "value", d["value"], "failed", d["failed_checks"], "spot", d["spot_check"])
for k in ("pcie_inclusive_all_ranks","c5_job","c5_job_one_process"):
    v=d.get(k,{}); print(k, {x: v.get(x) for x in ("all_ranks_GiBps","check","encode_ms","gather_ms","GBps_into_root","root_check","error")})'
