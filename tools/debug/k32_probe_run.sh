set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_protocol.py tests/test_ctc.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03b/tests.log 2>&1 || exit $?
tail -3 gpurun_out/r03b/tests.log
export WK_V=$PWD/esp32-wake-word_amd/build
timeout -k 10 200 python -u tools/debug/k32_probe.py bf16 4 > gpurun_out/r03b/probe_prod.log 2>&1 || exit $?
WAKEWORD_LIB=$WK_V/var_k32pad/libwakeword.so timeout -k 10 200 python -u tools/debug/k32_probe.py bf16 12 > gpurun_out/r03b/probe_k32pad.log 2>&1 || exit $?
WAKEWORD_LIB=$WK_V/var_k32dbg/libwakeword.so timeout -k 10 300 python -u tools/debug/k32_probe.py bf16 8 > gpurun_out/r03b/probe_k32dbg.log 2>&1 || exit $?
tail -2 gpurun_out/r03b/probe_*.log
