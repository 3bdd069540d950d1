set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mode_a.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b/gputest_fe.log 2>&1; rc=$?; tail -3 gpurun_out/r04b/gputest_fe.log; [ $rc -eq 0 ] || exit $rc
bash tools/debug/ab.sh base prod 2>&1 | tee gpurun_out/r04b/ab_fp32.txt
AB_ARGS="--precision bf16" bash tools/debug/ab.sh base prod 2>&1 | tee gpurun_out/r04b/ab_bf16.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r04b/gputest.log 2>&1; rc=$?; tail -5 gpurun_out/r04b/gputest.log; exit $rc
