# round 5: wave-cooperative near-tie re-scoring (rsw): CTC tests on it, then A/B + kernel stats
set -o pipefail
O=$PWD/gpurun_out/r05aa
mkdir -p $O
L=$PWD/variants/var_rsw/libwakeword.so
WAKEWORD_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -q -s --timeout 300 --timeout-method thread -k "ctc or config5" > $O/tests.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -20 $O/tests.log; exit $rc; }
tail -2 $O/tests.log; grep "config5 decisions" $O/tests.log | grep -v print | cut -c1-140
bash tools/debug/ctc_ab.sh rsw 2>&1 | tee $O/ab.txt
cd /tmp && export TMPDIR=/tmp
WAKEWORD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench_ctc.py" --no-cpu-baseline > "$O/prof.log" 2>&1 || exit $?
grep rescore $O/trace/run_kernel_stats.csv | cut -c1-40,100-200
