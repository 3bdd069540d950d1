set -o pipefail
mkdir -p gpurun_out/ab
WAKEWORD_LIB=$PWD/variants/var_ost/libwakeword.so timeout -k 10 120 python -u tools/debug/out_stamps.py > gpurun_out/ab/out_stamps.log 2>&1; rc=$?
tail -12 gpurun_out/ab/out_stamps.log; exit $rc
