#!/bin/bash
# C4's eager region alone vs in the full line (host submission per launch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4y}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c4 --steps 200 --warmup 5 --no-cpu --no-extras --no-configs > "$OUT/c4_alone.out" 2> "$OUT/c4_alone.err" || exit $?
python - "$OUT/c4_alone.out" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c4 alone:", d["value"], d["ms_per_step"], d["event_ms_per_step"], d["roofline"]["avg_kernel_ms"], d.get("region_host"))
PY
timeout -k 10 300 python tools/c4_ab.py > "$OUT/c4_ab.out" 2>&1 || exit $?
tail -3 "$OUT/c4_ab.out"
