#!/bin/bash
# Round 4, first GPU call: the copy-ordering test (current code), the same
# check against the pre-0b854e9 copy pattern (tools/ordering_revert.py
# variants) with and without the null-stream hook, and the N=2 bench
# rehearsal whose c5_job is now the C-ABI rank form.  Each step has its own
# time limit; a fault / abort / time-out ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r4a}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
OLD=cppserver_amd/_build/var/oldcopy/libwsg.so
OLDLB=tests/cpp/_build/var/libloopback_oldcopy.so
step ord_new 300 python -u -m pytest tests/test_gpu_c5.py -x -v --timeout 280 --timeout-method thread -k "copy_ordering"
step u32 200 python -u -m pytest tests/test_gpu_launch_shapes.py -x -v --timeout 120 --timeout-method thread -k "u32"
step ord_old_nospin 200 env WSG_LIB_PATH=$OLD WSG_RCCL_LIB=$OLDLB WSG_RANK_JOB=ordering python -u tests/mgpu_rank_job.py
step ord_old_spin 200 env WSG_LIB_PATH=$OLD WSG_RCCL_LIB=$OLDLB WSG_RANK_JOB=ordering WSG_TEST_NULL_SPIN_US=50000 python -u tests/mgpu_rank_job.py
step ord_oldprod_newlb_spin 200 env WSG_LIB_PATH=$OLD WSG_RCCL_LIB=tests/cpp/_build/libloopback_rccl.so WSG_RANK_JOB=ordering WSG_TEST_NULL_SPIN_US=50000 python -u tests/mgpu_rank_job.py
step ord_old_rccl_spin 200 env WSG_LIB_PATH=$OLD WSG_TEST_NULL_SPIN_US=50000 python -u tests/mgpu_rank_procs.py --ordering
step echo_prof_1c 120 tools/_build/bench_echo_prof per_read 1 1 1000 32 3
step echo_prof_100c 120 tools/_build/bench_echo_prof per_read 100 4 1000 32 3
step echo_ref_1c 120 tools/_build/bench_echo_ref 1 1 1000 32 3
step c3_enc_diag 300 python -u tools/c3_enc_diag.py
step fan_many_ab 200 python -u tools/fan_many_ab.py
step bench_n2_test 400 python -u -m pytest tests/test_gpu_c5.py -x -v --timeout 380 --timeout-method thread -k "bench_n2"
if [ "${SKIP_BENCH:-0}" != "1" ]; then
step bench_n2 900 env WSG_BENCH_SHARE_DEVICES=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5
fi
echo "== done"
