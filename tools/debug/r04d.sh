set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r04d/gputest.log 2>&1; rc=$?; tail -4 gpurun_out/r04d/gputest.log; [ $rc -eq 0 ] || exit $rc
bash tools/debug/ab.sh base prod 2>&1 | tee gpurun_out/r04d/ab_fp32.txt
timeout -k 10 400 bash tools/pmc_census.sh gpurun_out/r04d/census > gpurun_out/r04d/census.log 2>&1 && python3 tools/pmc_census.py gpurun_out/r04d/census --json gpurun_out/r04d/census.json > gpurun_out/r04d/census.txt; cat gpurun_out/r04d/census.txt
