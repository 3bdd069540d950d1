set -o pipefail
mkdir -p gpurun_out/r03d
export WK_V=$PWD/esp32-wake-word_amd/build
for v in k32chk k32gap k32pool; do
WAKEWORD_LIB=$WK_V/var_$v/libwakeword.so timeout -k 10 200 python -u tools/debug/k32_probe.py bf16 4 > gpurun_out/r03d/probe_$v.log 2>&1 || exit $?
done
for v in k32chk k32gap k32pool; do echo == $v; grep -h "^rep\|classif\|bounds" gpurun_out/r03d/probe_$v.log; done
