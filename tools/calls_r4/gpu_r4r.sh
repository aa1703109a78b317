#!/bin/bash
# Full GPU suite + smoke after the round-4 lane / host-path changes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4r}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== suite $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/suite.log" 2>&1
rc=$?
tail -5 "$OUT/suite.log"
[ $rc -ne 0 ] && exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
rc=$?
tail -2 "$OUT/smoke.log"
[ $rc -ne 0 ] && exit $rc
echo "== sampled echo $(date +%T)"
WSG_SAMPLER=100 WSG_SAMPLER_OUT="$OUT/samp_gpu_1c.txt" timeout -k 10 60 tools/_build/bench_echo_samp per_read 1 1 1000 32 5 > "$OUT/samp_gpu_1c.log" 2>&1 || exit $?
tail -1 "$OUT/samp_gpu_1c.log"
WSG_SAMPLER=100 WSG_SAMPLER_OUT="$OUT/samp_host_1c.txt" timeout -k 10 60 tools/_build/echo_hostonly_samp per_read 1 1 1000 32 5 > "$OUT/samp_host_1c.log" 2>&1 || exit $?
tail -1 "$OUT/samp_host_1c.log"
