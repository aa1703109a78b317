set -o pipefail
O=gpurun_out/r2d; mkdir -p $O
V=cppserver_amd/_build/var
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { echo TESTS_FAILED; tail -40 $O/gputests.txt; exit 1; }
for m in per_read tick per_call; do timeout -k 10 60 tools/_build/bench_echo $m 1 1 1000 32 3 >> $O/echo.txt 2>&1 || { echo ECHO_FAILED $m; tail $O/echo.txt; exit 1; }; done
timeout -k 10 60 tools/_build/bench_echo per_read 100 4 1000 32 3 >> $O/echo.txt 2>&1 || { echo ECHO100_FAILED; tail $O/echo.txt; exit 1; }
timeout -k 10 60 tools/_build/bench_echo tick 100 1 1000 32 3 >> $O/echo.txt 2>&1 || { echo ECHOT_FAILED; tail $O/echo.txt; exit 1; }
CFG=c5 timeout -k 10 200 python -u tools/tune_enc.py cppserver_amd/_build/libwsg.so $V/encsc1/libwsg.so > $O/tune_enc_c5.txt 2>&1 || { echo TUNEENC_FAILED; tail $O/tune_enc_c5.txt; exit 1; }
CFG=c3 timeout -k 10 200 python -u tools/tune_enc.py cppserver_amd/_build/libwsg.so $V/encsc1/libwsg.so > $O/tune_enc_c3.txt 2>&1 || { echo TUNEENC3_FAILED; exit 1; }
CFG=c4 timeout -k 10 200 python -u tools/tune_enc.py cppserver_amd/_build/libwsg.so $V/fannt/libwsg.so > $O/tune_fan.txt 2>&1 || { echo TUNEFAN_FAILED; exit 1; }
echo ALL_OK
