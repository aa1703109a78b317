set -o pipefail
O=gpurun_out/r2g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.txt; exit 1; }
for l in "tx 256 64 32 0 3" "rx 256 64 32 0 3"; do timeout -k 10 120 tools/_build/bench_batch $l >> $O/batch.txt 2>&1 || { echo BATCH_FAILED; exit 1; }; done
timeout -k 10 60 tools/_build/bench_echo per_read 1 1 1000 32 3 >> $O/echo.txt 2>&1 || { echo ECHO_FAILED; exit 1; }
timeout -k 10 120 tools/_build/membench 0 wpattern > $O/wpattern.txt 2>&1 || { echo WP_FAILED; exit 1; }
timeout -k 10 120 tools/_build/membench 0 write > $O/write.txt 2>&1 || { echo W_FAILED; exit 1; }
echo ALL_OK
