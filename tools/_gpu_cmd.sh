mkdir -p gpurun_out/g12
L=cppserver_amd/_build
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -x -k "fanout" > gpurun_out/g12/t.log 2>&1 || exit $?
CFG=c4 REPS=7 timeout -k 10 200 python tools/tune_enc.py $L/var/pieces/libwsg.so $L/libwsg.so $L/var/fu2/libwsg.so $L/var/fu8/libwsg.so > gpurun_out/g12/c4.log 2>&1
CFG=c4 LEN=1000 KEYS=20000 timeout -k 10 200 python tools/tune_enc.py $L/libwsg.so $L/var/fu2/libwsg.so $L/var/fu8/libwsg.so >> gpurun_out/g12/c4.log 2>&1
