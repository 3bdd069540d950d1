set -o pipefail
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -4 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py > $O/bench_fp32.log 2>&1 || exit $?
tail -1 $O/bench_fp32.log | cut -c1-400
timeout -k 10 180 python bench.py --no-cpu-baseline --precision bf16 --batch 131072 > $O/bench_bf16_131k.log 2>&1 || exit $?
tail -1 $O/bench_bf16_131k.log | cut -c1-300
timeout -k 10 400 bash tools/pmc_census.sh $O/census > $O/census.log 2>&1 && python3 tools/pmc_census.py $O/census --json $O/census.json > $O/census.txt; cat $O/census.txt
