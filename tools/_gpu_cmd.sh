set -u
mkdir -p gpurun_out/g3
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/g3/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/g3/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 tools/_build/membench 0 write > gpurun_out/g3/write.log 2>&1 || exit $?
cat gpurun_out/g3/write.log
