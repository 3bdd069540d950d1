set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -k decision_parity -s -q --timeout 200 --timeout-method thread > $O/decision.log 2>&1; grep "config5 decisions" $O/decision.log
timeout -k 10 240 python bench.py > $O/bench_fp32.log 2>&1 || exit $?
tail -1 $O/bench_fp32.log | cut -c1-600
timeout -k 10 180 python bench.py --no-cpu-baseline --precision bf16 --batch 131072 > $O/bench_bf16_131k.log 2>&1 || exit $?
tail -1 $O/bench_bf16_131k.log | cut -c1-300
bash tools/debug/ab.sh base div div2 div2slds 2>&1 | tee $O/ab.txt
timeout -k 10 400 bash tools/pmc_census.sh $O/census > $O/census.log 2>&1 && python3 tools/pmc_census.py $O/census --json $O/census.json > $O/census.txt; cat $O/census.txt
for x in 0 1 2; do
  WAKEWORD_LIB=$PWD/variants/var_exp/libwakeword.so WAKEWORD_FUSED_EXP=$x timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/roles_$x.log 2>&1 || exit $?
  python -c "import json;d=json.loads(open('$O/roles_$x.log').read().strip().splitlines()[-1]);print('exp=$x', d['roofline']['launch_ms'], 'ms', round(d['value']/1e6,3), 'M win/s')"
done
