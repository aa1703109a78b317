set -e
mkdir -p gpurun_out/fan6
L=cppserver_amd/_build
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -x -k "fanout" > gpurun_out/fan6/t.log 2>&1
CFG=c4 REPS=7 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so $L/var/fan3/libwsg.so > gpurun_out/fan6/c4.log 2>&1
CFG=c4 LEN=16 KEYS=100000 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so >> gpurun_out/fan6/c4.log 2>&1
CFG=c4 LEN=1000 KEYS=20000 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so >> gpurun_out/fan6/c4.log 2>&1
