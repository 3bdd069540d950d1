set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r04b/gputest.log 2>&1; rc=$?; tail -8 gpurun_out/r04b/gputest.log; [ $rc -eq 0 ] || exit $rc
bash tools/debug/ab.sh base prod 2>&1 | tee gpurun_out/r04b/ab_fp32.txt
AB_ARGS="--precision bf16" bash tools/debug/ab.sh base prod 2>&1 | tee gpurun_out/r04b/ab_bf16.txt
