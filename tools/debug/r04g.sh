set -o pipefail
O=$PWD/gpurun_out/r04g
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -3 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -k decision_parity -s -q --timeout 200 --timeout-method thread > $O/decision.log 2>&1; grep "config5 decisions" $O/decision.log
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_fp32.log 2>&1 || exit $?
tail -1 $O/bench_fp32.log | cut -c1-300
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "counters listed rc=$?"
timeout -k 10 400 bash tools/pmc_census.sh $O/census > $O/census.log 2>&1 && python3 tools/pmc_census.py $O/census --json $O/census.json > $O/census.txt; cat $O/census.txt
for x in 1 2; do
  WAKEWORD_LIB=$PWD/variants/var_exp/libwakeword.so WAKEWORD_FUSED_EXP=$x timeout -k 10 400 bash tools/pmc_census.sh $O/census_exp$x > $O/census_exp$x.log 2>&1 && python3 tools/pmc_census.py $O/census_exp$x --json $O/census_exp$x.json > $O/census_exp$x.txt; echo "== exp $x"; cat $O/census_exp$x.txt
done
bash tools/debug/ab.sh base div2 edge edgeg1 edgeg1pk 2>&1 | tee $O/ab.txt
