#!/bin/bash
# PMC passes on the GPU box: FETCH_SIZE and WRITE_SIZE in separate runs (TCC
# slots), for the bench (C2) and for membench's calibration kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 1 --no-cpu --no-extras ${BENCH_ARGS:-}"
for c in FETCH_SIZE WRITE_SIZE; do
    echo "== bench $c"
    timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/bench_$c" -o run --output-format csv -- $B > "$OUT/bench_$c.log" 2>&1 || exit $?
    echo "== membench $c"
    timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/mem_$c" -o run --output-format csv -- tools/_build/membench 1024 calib > "$OUT/mem_$c.log" 2>&1 || exit $?
done
echo "== done"
