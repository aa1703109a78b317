#!/bin/bash
# Everything profiles/ needs for one round, in one GPU call: the bench line,
# the rocprofv3 kernel-trace summary of the same command, and PMC passes
# (FETCH_SIZE, WRITE_SIZE separately) with membench calibration.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-r1}
OUT=gpurun_out/art_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python bench.py ${STEPS:+--steps $STEPS}"   # bench.py defaults unless STEPS is set
echo "== bench"
timeout -k 10 600 $B > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
tail -1 "$OUT/bench.json"
echo "== kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $B --no-cpu --no-extras > "$OUT/trace.log" 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $c"
    timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/pmc/bench_$c" -o run --output-format csv -- $B --steps 5 --no-cpu --no-extras > "$OUT/pmc_$c.log" 2>&1 || exit $?
    timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/pmc/mem_$c" -o run --output-format csv -- tools/_build/membench 1024 calib > "$OUT/pmcm_$c.log" 2>&1 || exit $?
done
for c in c3 c4 c5; do
    echo "== bench $c"
    timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-extras > "$OUT/bench_$c.json" 2>/dev/null || exit $?
    tail -1 "$OUT/bench_$c.json"
done
echo "== done"
