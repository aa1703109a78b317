#!/bin/bash
# One round's evidence for profiles/$ROUND (ROUND=r4 ...), in one GPU call:
#  * the driver's own command (python bench.py --steps 20 --warmup 5): the
#    C2 headline line with its c3 / c4 / c5 objects;
#  * the same command under rocprofv3 --kernel-trace --marker-trace --stats
#    (bench.py marks every leg's timed region with a roctx range, so
#    tools/trace_split.py assigns each kernel launch to its leg);
#  * HBM traffic from PMC, FETCH_SIZE and WRITE_SIZE in separate passes (the
#    guide's rule), one bench process per config (kernel names repeat across
#    configs), plus membench's known-byte kernels for the FETCH_SIZE
#    calibration in the same passes.
# PMC=1 BENCH=0: the counter passes only (collect them first, so that the
# bench line of a second call carries this round's traffic); BENCH=1 PMC=0:
# the line and its trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:?set ROUND, e.g. ROUND=r4}
OUT=gpurun_out/art_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name, timeout, command...
    local name=$1 t=$2
    shift 2
    echo "== $name $(date +%T)" | tee -a "$OUT/progress.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err" || { echo "FAILED $name rc=$?" | tee -a "$OUT/progress.log"; exit 1; }
}
if [ "${BENCH:-1}" = 1 ]; then
    run bench 600 python bench.py --steps 20 --warmup 5
    # the same command; its host-side child legs (echo, multicast, session
    # batches: no kernel of the GPU legs) are skipped, tracing them takes minutes
    export WSG_BENCH_HOST_LEGS=0
    run trace 900 rocprofv3 --kernel-trace --marker-trace --stats -d "$OUT/trace" -o run \
        --output-format csv -- python bench.py --steps 20 --warmup 5
    unset WSG_BENCH_HOST_LEGS
fi
[ "${PMC:-1}" = 1 ] && for c in ${CFGS:-c2 c3 c4 c5}; do
    for k in FETCH_SIZE WRITE_SIZE; do
        run "pmc_${c}_$k" 300 rocprofv3 --pmc $k -d "$OUT/pmc_${c}_$k" -o run --output-format csv -- \
            python bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-extras --no-configs
    done
done
[ "${PMC:-1}" = 1 ] && for k in FETCH_SIZE WRITE_SIZE; do
    run "pmc_calib_$k" 300 rocprofv3 --pmc $k -d "$OUT/pmc_calib_$k" -o run --output-format csv -- \
        tools/_build/membench 1024 calib
done
echo "== done $(date +%T)" | tee -a "$OUT/progress.log"
