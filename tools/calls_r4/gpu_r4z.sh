#!/bin/bash
# C4 inside the line: with and without the extras legs before the configs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4z}
mkdir -p "$OUT"
export TMPDIR=/tmp
show() {
python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c4 = d["c4"]
print(sys.argv[1], "c4", c4["value"], c4["ms_per_step"], c4["event_ms_per_step"], c4["warmup"], "c3", d["c3"]["value"], "c5", d["c5"]["value"])
PY
}
WSG_BENCH_HOST_LEGS=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > "$OUT/line_extras.out" 2> "$OUT/line_extras.err" || exit $?
show "$OUT/line_extras.out"
WSG_BENCH_HOST_LEGS=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu --no-extras > "$OUT/line_noextras.out" 2> "$OUT/line_noextras.err" || exit $?
show "$OUT/line_noextras.out"
