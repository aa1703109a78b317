set -o pipefail
O=gpurun_out/r2f; mkdir -p $O
V=cppserver_amd/_build/var
ROT=2 REPS=11 timeout -k 10 300 python -u tools/tune.py 48@$V/head/libwsg.so 48 48@$V/sc1/libwsg.so 48@$V/buf/libwsg.so 48@$V/bufsc1/libwsg.so 56@$V/bufsc1/libwsg.so > $O/tune_c2.txt 2>&1 || { echo TUNE2_FAILED; tail $O/tune_c2.txt; exit 1; }
RAGGED=128,65536 FRAMES=65536 REPS=5 timeout -k 10 200 python -u tools/tune.py 48 48@$V/bufsc1/libwsg.so > $O/tune_c3.txt 2>&1 || { echo TUNE3_FAILED; exit 1; }
echo ALL_OK
