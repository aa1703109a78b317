#!/bin/bash
# k_decode with the batch's tail in 4 KiB tiles (WSG_DEC_TAIL_PCT) against
# the round's kernel: parity first (C2 / C3 full size, decode edge cases,
# 300-seed fuzz) on the variants, then C2 and C3 bench legs interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r6u}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=$PWD/cppserver_amd/_build/var
for v in ${PARITY:-dt35 dt50}; do
  WSG_LIB_PATH=$V/$v/libwsg.so WSG_FUZZ_SEEDS=300 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py -k "decode or c2 or c3 or garbage or truncat or length or fuzz_encode" > "$OUT/parity_$v.log" 2>&1 || { echo "parity $v rc=$?"; tail -30 "$OUT/parity_$v.log"; exit 1; }
  echo "parity $v: $(tail -n 1 "$OUT/parity_$v.log")"
done
: > "$OUT/ab.log"
for round in 1 2 3; do
  for v in ${VARIANTS:-prev dt0 dt25 dt35 dt50}; do
    for cfg in c2 c3; do
      steps=50; [ $cfg = c3 ] && steps=20
      r=$(WSG_LIB_PATH=$V/$v/libwsg.so timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 10 --no-cpu --no-extras --no-configs 2>/dev/null | tail -n 1) || { echo "bench $v $cfg failed"; exit 1; }
      echo "$r" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); rf=d['roofline']
h=[(x['kernel'],x['frac'],x['avg_kernel_ms']) for x in rf.get('halves',[rf])]
print('$v $cfg', d['value'], h, d['spot_check'])" >> "$OUT/ab.log"
    done
  done
done
cat "$OUT/ab.log"
