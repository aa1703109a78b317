mkdir -p gpurun_out/g13
WSG_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/g13/dist2.json 2> gpurun_out/g13/dist2.err; echo "rc=$?" >> gpurun_out/g13/dist2.err
timeout -k 10 600 python -m pytest tests/test_gpu_rx_batch.py -q -x -k repeated > gpurun_out/g13/rx.log 2>&1; echo "rc=$?" >> gpurun_out/g13/rx.log
