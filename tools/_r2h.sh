set -o pipefail
O=gpurun_out/r2h; mkdir -p $O
V=cppserver_amd/_build/var
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x -k "fanout" --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/t.log; exit 1; }
CFG=c4 REPS=9 timeout -k 10 200 python -u tools/tune_enc.py $V/fanold/libwsg.so $V/fanpipe0/libwsg.so $V/fanpipe1/libwsg.so cppserver_amd/_build/libwsg.so > $O/c4.txt 2>&1 || { echo C4_FAILED; tail $O/c4.txt; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --steps 50 --warmup 3 --no-cpu > $O/bench_c4.json 2> $O/bench_c4.err || { echo B4_FAILED; tail $O/bench_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --messages 16 --steps 20 --warmup 3 --no-cpu > $O/bench_c4x16.json 2> $O/bench_c4x16.err || { echo B16_FAILED; tail $O/bench_c4x16.err; exit 1; }
echo ALL_OK
