mkdir -p gpurun_out/ab
for c in c5 c3; do
CFG=$c REPS=5 timeout -k 10 300 python tools/tune_enc.py cppserver_amd/_build/var/old/libwsg.so cppserver_amd/_build/libwsg.so > gpurun_out/ab/enc_$c.log 2>&1 || exit $?
cat gpurun_out/ab/enc_$c.log
done
