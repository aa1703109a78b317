#!/bin/bash
# Round-2 evidence for profiles/r2, in one GPU call: for every BASELINE
# config bench.py runs (c2 headline, c3, c4, c4 x 16 messages, c5 one-GPU
# shard) the bench line, the rocprofv3 kernel trace (--kernel-trace --stats)
# of the same command, and HBM traffic from PMC (FETCH_SIZE and WRITE_SIZE in
# separate passes, the guide's rule), plus membench's known-byte kernels for
# the FETCH_SIZE calibration in the same passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/art_r2
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name, timeout, command...
    local name=$1 t=$2
    shift 2
    echo "== $name $(date +%T)" | tee -a "$OUT/progress.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "FAILED $name rc=$?" | tee -a "$OUT/progress.log"; exit 1; }
}
declare -A ARGS=(
    [c2]="--config c2"
    [c3]="--config c3"
    [c4]="--config c4"
    [c4x16]="--config c4 --messages 16"
    [c5]="--config c5"
)
declare -A STEPS=([c2]=200 [c3]=10 [c4]=50 [c4x16]=20 [c5]=10)
for c in ${CFGS:-c2 c3 c4 c4x16 c5}; do
    run "bench_$c" 600 python bench.py ${ARGS[$c]} --steps ${STEPS[$c]} --warmup 3
    run "trace_$c" 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$c" -o run --output-format csv -- \
        python bench.py ${ARGS[$c]} --steps ${STEPS[$c]} --warmup 3 --no-cpu --no-extras
    for k in FETCH_SIZE WRITE_SIZE; do
        run "pmc_${c}_$k" 300 rocprofv3 --pmc $k -d "$OUT/pmc_${c}_$k" -o run --output-format csv -- \
            python bench.py ${ARGS[$c]} --steps 5 --warmup 1 --no-cpu --no-extras
    done
done
[ "${CALIB:-1}" = 1 ] && for k in FETCH_SIZE WRITE_SIZE; do
    run "pmc_calib_$k" 300 rocprofv3 --pmc $k -d "$OUT/pmc_calib_$k" -o run --output-format csv -- \
        tools/_build/membench 1024 calib
done
echo "== done $(date +%T)" | tee -a "$OUT/progress.log"
