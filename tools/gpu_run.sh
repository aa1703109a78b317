#!/bin/bash
# Runner for the GPU box: GPU tests, smoke, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit.  A test assertion failure (pytest
# rc 1) does not stop the run; any other non-zero status (fault, abort,
# timeout) ends it there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    tail -4 "$OUT/$name.log"
    return $rc
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
    step pytest_gpu 900 python -m pytest tests -m gpu -x -q
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
step bench 600 python bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:-} || exit $?
if [ "${SKIP_PROF:-0}" != "1" ]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu --no-extras ${BENCH_ARGS:-} || exit $?
fi
echo "== done"
