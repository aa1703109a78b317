#!/bin/bash
# GPU tests, then C2 frame-size sweep (tools/tune.py) and the C3/C4/C5 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
    timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_perf.log 2>&1
    rc=$?; tail -2 gpurun_out/pytest_perf.log
    [ $rc -le 1 ] || exit $rc
fi
for cfg in ${SWEEP:-"1 268435456" "4096 65536" "16384 16384" "65536 4096"}; do
    set -- $cfg
    echo -n "frames=$1 size=$2: "
    FRAMES=$1 SIZE=$2 REPS=5 EVERY=8 timeout -k 10 200 python tools/tune.py ${BPC:-32} | tail -1 || exit 1
done
for c in ${CONFIGS:-c3 c4 c5}; do
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-extras 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"$c\", d[\"value\"], \"GiB/s  step\", d[\"ms_per_step\"], \"ms  kernel\", d[\"roofline\"][\"avg_kernel_ms\"], \"ms\", d[\"roofline\"][\"achieved\"], \"GB/s\")" || exit 1
done
