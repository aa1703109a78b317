#!/bin/bash
# Sweep the unmask grid size (blocks per CU) on the C2 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in ${BPCS:-4 6 8 12 16 32 64}; do
    echo -n "bpc=$b "
    WSG_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu --no-extras ${BENCH_ARGS:-} 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_kernel_ms'], d['roofline']['achieved'])" || exit $?
done
