set -o pipefail
mkdir -p gpurun_out/k32
export WKL=$PWD/esp32-wake-word_amd/build/var_k32/libwakeword.so
WAKEWORD_LIB=$WKL timeout -k 10 200 python tools/debug/race_probe.py bf16 12 > gpurun_out/k32/race_bf16.log 2>&1 || exit $?
WAKEWORD_LIB=$WKL timeout -k 10 200 python tools/debug/race_probe.py bf16x3 12 > gpurun_out/k32/race_bf16x3.log 2>&1 || exit $?
AB_ARGS="--precision bf16" bash tools/debug/ab.sh prod k32 || exit $?
AB_ARGS="--precision bf16x3" bash tools/debug/ab.sh prod k32 || exit $?
