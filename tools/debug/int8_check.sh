#!/bin/bash
# int8 path on the GPU box: its tests (MFMA kernel), then the call-surface bench
# with the MFMA kernel and with the VALU checking kernel (WAKEWORD_INT8_VALU=1).
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
mkdir -p gpurun_out/i8
timeout -k 10 300 python -u -m pytest tests/test_gpu_int8.py tests/test_device_detector.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/i8/tests.log 2>&1
rc=$?; tail -3 gpurun_out/i8/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_surfaces.py --cpu-clips 0 > gpurun_out/i8/surf_mfma.log 2>&1 || exit $?
WAKEWORD_INT8_VALU=1 timeout -k 10 300 python bench_surfaces.py --cpu-clips 0 > gpurun_out/i8/surf_valu.log 2>&1 || exit $?
grep -h '^{' gpurun_out/i8/surf_mfma.log gpurun_out/i8/surf_valu.log | python -c "
import sys, json
for l in sys.stdin: d = json.loads(l); print(d['wk_cnn_int8'], d['wk_cnn_fp32'])"
