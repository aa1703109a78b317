set -o pipefail
O=gpurun_out/r2b; mkdir -p $O
V=cppserver_amd/_build/var
timeout -k 10 300 python -u bench.py --config c4 --steps 50 --warmup 5 > $O/bench_c4.json 2> $O/bench_c4.err || { echo C4_FAILED; tail -20 $O/bench_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --messages 16 --steps 20 --warmup 3 > $O/bench_c4x16.json 2> $O/bench_c4x16.err || { echo C4M_FAILED; tail -20 $O/bench_c4x16.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err || { echo C5_FAILED; tail -20 $O/bench_c5.err; exit 1; }
WSG_BENCH_BACKEND=gloo WSG_C5_FRAMES=65536 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo N2_FAILED; tail -20 $O/bench_n2_gloo.err; exit 1; }
CFG=c4 timeout -k 10 200 python -u tools/tune_enc.py cppserver_amd/_build/libwsg.so $V/fansc1/libwsg.so > $O/tune_fan.txt 2>&1 || { echo TUNEFAN_FAILED; exit 1; }
RAGGED=128,65536 FRAMES=65536 REPS=5 timeout -k 10 200 python -u tools/tune.py 48@$V/head/libwsg.so 48 > $O/tune_c3.txt 2>&1 || { echo TUNE3_FAILED; exit 1; }
FRAMES=1048576 SIZE=32 REPS=5 timeout -k 10 200 python -u tools/tune.py 48@$V/head/libwsg.so 48 > $O/tune_32.txt 2>&1 || { echo TUNE32_FAILED; exit 1; }
echo ALL_OK
