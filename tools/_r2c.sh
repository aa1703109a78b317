set -o pipefail
O=gpurun_out/r2c; mkdir -p $O
V=cppserver_amd/_build/var
CFG=c4 timeout -k 10 200 python -u tools/tune_enc.py cppserver_amd/_build/libwsg.so $V/fansc1/libwsg.so > $O/tune_fan.txt 2>&1 || { echo TUNEFAN_FAILED; tail $O/tune_fan.txt; exit 1; }
RAGGED=128,65536 FRAMES=65536 REPS=5 timeout -k 10 200 python -u tools/tune.py 48@$V/head/libwsg.so 48 > $O/tune_c3.txt 2>&1 || { echo TUNE3_FAILED; tail $O/tune_c3.txt; exit 1; }
FRAMES=1048576 SIZE=32 REPS=5 timeout -k 10 200 python -u tools/tune.py 48@$V/head/libwsg.so 48 > $O/tune_32.txt 2>&1 || { echo TUNE32_FAILED; exit 1; }
ROT=2 REPS=9 timeout -k 10 200 python -u tools/tune.py 48@$V/head/libwsg.so 48 > $O/tune_c2.txt 2>&1 || { echo TUNE2_FAILED; exit 1; }
echo ALL_OK
