#!/bin/bash
# CTC tests + config-5 bench (fp16, fp32) on the GPU box.
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_ctc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ctc_tests.log 2>&1
tail -2 gpurun_out/ctc_tests.log
timeout -k 10 200 python -u bench_ctc.py > gpurun_out/ctc_bench16.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_ctc.py --precision fp32 > gpurun_out/ctc_bench32.log 2>&1 || exit 1
tail -1 gpurun_out/ctc_bench16.log; tail -1 gpurun_out/ctc_bench32.log
