set -o pipefail
mkdir -p gpurun_out/r2a
O=gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.txt 2>&1 || { echo TESTS_FAILED; tail -30 $O/gputests.txt; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { echo C2_FAILED; tail -20 $O/bench_c2.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 3 > $O/bench_c3.json 2> $O/bench_c3.err || { echo C3_FAILED; tail -20 $O/bench_c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --steps 50 --warmup 5 > $O/bench_c4.json 2> $O/bench_c4.err || { echo C4_FAILED; tail -20 $O/bench_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --messages 16 --steps 20 --warmup 3 > $O/bench_c4x16.json 2> $O/bench_c4x16.err || { echo C4M_FAILED; tail -20 $O/bench_c4x16.err; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err || { echo C5_FAILED; tail -20 $O/bench_c5.err; exit 1; }
WSG_BENCH_BACKEND=gloo WSG_C5_FRAMES=65536 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo N2_FAILED; tail -20 $O/bench_n2_gloo.err; exit 1; }
echo ALL_OK
