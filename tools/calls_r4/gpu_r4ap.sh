#!/bin/bash
# The driver's N = 4 command, rehearsed with both ranks on the one GPU (RCCL over sockets), default legs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4aj}
mkdir -p "$OUT"
export TMPDIR=/tmp
export WSG_BENCH_SHARE_DEVICES=1
echo "== n4 $(date +%T)"
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29542 \
    bench.py --gpus 4 --steps 20 --warmup 5 > "$OUT/n4.out" 2> "$OUT/n4.err"
rc=$?
echo "rc=$rc $(date +%T)"
grep "^{" "$OUT/n4.out" | tail -1 | cut -c1-1500
tail -5 "$OUT/n4.err"
exit $rc
