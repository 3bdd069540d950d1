#!/bin/bash
# K = 32 bf16 MFMA with the eager DCT off: is the clip-4 corruption tied to the
# eager path?  race_probe (feature-dump build, 12 repeats) + A/B timing.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
mkdir -p gpurun_out/k32ne
WAKEWORD_LIB=$R/esp32-wake-word_amd/build/var_k32ne/libwakeword.so timeout -k 10 200 python tools/debug/race_probe.py bf16 12 > gpurun_out/k32ne/race_bf16.log 2>&1 || exit $?
WAKEWORD_LIB=$R/esp32-wake-word_amd/build/var_k32ne/libwakeword.so timeout -k 10 200 python tools/debug/race_probe.py bf16x3 12 > gpurun_out/k32ne/race_bf16x3.log 2>&1 || exit $?
AB_ARGS="--precision bf16" bash tools/debug/ab.sh prod ne k32ne || exit $?
