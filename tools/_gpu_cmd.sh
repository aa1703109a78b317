set -e
mkdir -p gpurun_out/g5
L=cppserver_amd/_build
set +e
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/g5/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/g5/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
CFG=c4 REPS=7 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so $L/var/fan3/libwsg.so > gpurun_out/g5/c4.log 2>&1
CFG=c4 LEN=16 KEYS=100000 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so >> gpurun_out/g5/c4.log 2>&1
CFG=c4 LEN=1000 KEYS=20000 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so >> gpurun_out/g5/c4.log 2>&1
timeout -k 10 120 tools/_build/membench 256 map > gpurun_out/g5/map.log 2>&1
timeout -k 10 300 tools/_build/bench_batch rx 1024 4 65536 16384 3 > gpurun_out/g5/batch.log 2>&1
timeout -k 10 300 tools/_build/bench_batch tx 1024 4 65536 0 3 >> gpurun_out/g5/batch.log 2>&1
timeout -k 10 300 tools/_build/bench_batch rx 4096 8 32 0 3 >> gpurun_out/g5/batch.log 2>&1
timeout -k 10 300 tools/_build/bench_batch tx 4096 8 32 0 3 >> gpurun_out/g5/batch.log 2>&1
