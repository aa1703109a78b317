set -e
mkdir -p gpurun_out/g4
L=cppserver_amd/_build
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -x -k "fanout" > gpurun_out/g4/t.log 2>&1
CFG=c4 REPS=7 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so $L/var/fan3/libwsg.so > gpurun_out/g4/c4.log 2>&1
CFG=c4 LEN=16 KEYS=100000 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so >> gpurun_out/g4/c4.log 2>&1
CFG=c4 LEN=1000 KEYS=20000 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so >> gpurun_out/g4/c4.log 2>&1
timeout -k 10 120 tools/_build/membench 256 map > gpurun_out/g4/map.log 2>&1
timeout -k 10 300 tools/_build/bench_batch rx 1024 4 65536 16384 3 > gpurun_out/g4/batch.log 2>&1
timeout -k 10 300 tools/_build/bench_batch tx 1024 4 65536 0 3 >> gpurun_out/g4/batch.log 2>&1
timeout -k 10 300 tools/_build/bench_batch rx 4096 8 32 0 3 >> gpurun_out/g4/batch.log 2>&1
timeout -k 10 300 tools/_build/bench_batch tx 4096 8 32 0 3 >> gpurun_out/g4/batch.log 2>&1
