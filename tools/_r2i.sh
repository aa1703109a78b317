set -o pipefail
O=gpurun_out/r2l; mkdir -p $O
V=cppserver_amd/_build/var
export TMPDIR=/tmp
timeout -k 10 60 tools/_build/membench 0 empty > $O/empty.txt 2>&1 || { echo EMPTY_FAILED; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/p_empty -o run --output-format csv -- tools/_build/membench 0 empty > $O/p_empty.txt 2>&1 || { echo PE_FAILED; exit 1; }
for v in var/fannew112 .; do
  n=$(basename $v)
  CFG=c4 REPS=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $O/q_$n -o run --output-format csv -- python3 -u tools/tune_enc.py cppserver_amd/_build/$v/libwsg.so > $O/q_$n.txt 2>&1 || { echo Q_FAILED $v; tail $O/q_$n.txt; exit 1; }
done
echo ALL_OK
