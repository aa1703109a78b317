#!/bin/bash
# Where the one-client echo's time goes on the current tree (tools/echo_prof.cpp): per-call host framing, GPU passes, flushes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r5t}
mkdir -p "$OUT"
export TMPDIR=/tmp
for leg in "per_read 1 1" "per_read 100 4" "tick 100 1"; do
  timeout -k 10 60 tools/_build/bench_echo_prof $leg 1000 32 2 > "$OUT/prof_${leg// /_}.log" 2>&1 || { echo "fail $leg"; tail -5 "$OUT/prof_${leg// /_}.log"; exit 1; }
  echo "== $leg"; cat "$OUT/prof_${leg// /_}.log"
done
