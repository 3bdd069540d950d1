set -o pipefail
mkdir -p gpurun_out/ab
WAKEWORD_LIB=$PWD/variants/var_st/libwakeword.so timeout -k 10 120 python -u tools/debug/gru_stamps.py > gpurun_out/ab/gru_stamps.log 2>&1; rc=$?
cat gpurun_out/ab/gru_stamps.log | tail -20; exit $rc
