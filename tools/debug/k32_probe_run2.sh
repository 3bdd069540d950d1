set -o pipefail
mkdir -p gpurun_out/r03c
export WK_V=$PWD/esp32-wake-word_amd/build
WAKEWORD_LIB=$WK_V/var_k32noepi/libwakeword.so timeout -k 10 200 python -u tools/debug/k32_probe.py bf16 6 > gpurun_out/r03c/probe_k32noepi.log 2>&1 || exit $?
WAKEWORD_LIB=$WK_V/var_k16dbg/libwakeword.so timeout -k 10 200 python -u tools/debug/k32_probe.py bf16 6 > gpurun_out/r03c/probe_k16dbg.log 2>&1 || exit $?
grep -h "^rep\|classif" gpurun_out/r03c/*.log
