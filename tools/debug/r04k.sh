set -o pipefail
O=$PWD/gpurun_out/r04k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/ctc_tests.log 2>&1; rc=$?; tail -2 $O/ctc_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/debug/ctc_ab.sh lmbase lmwin gruds 2>&1 | tee $O/ctc_ab.txt
