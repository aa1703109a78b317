set -o pipefail
O=gpurun_out/r2e; mkdir -p $O
V=cppserver_amd/_build/var
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "c3_roundtrip or host_pipeline or wire_cap" --timeout 250 --timeout-method thread > $O/c3test.txt 2>&1 || { echo C3TEST_FAILED; tail -30 $O/c3test.txt; exit 1; }
ROT=2 REPS=9 timeout -k 10 300 python -u tools/tune.py 48@$V/head/libwsg.so 48 48@$V/infolast/libwsg.so 48@$V/noinfo/libwsg.so 48@$V/diag5/libwsg.so 48@$V/u8/libwsg.so 40 56 64 > $O/tune_c2.txt 2>&1 || { echo TUNE2_FAILED; tail $O/tune_c2.txt; exit 1; }
timeout -k 10 120 tools/_build/membench 256 policy > $O/policy.txt 2>&1 || { echo POLICY_FAILED; exit 1; }
echo ALL_OK
