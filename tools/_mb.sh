mkdir -p gpurun_out/mb
for m in 256 2048; do
timeout -k 10 120 tools/_build/membench $m explore > gpurun_out/mb/explore_$m.log 2>&1 || exit $?
echo "== $m"; grep -E "copy delta" gpurun_out/mb/explore_$m.log
done
