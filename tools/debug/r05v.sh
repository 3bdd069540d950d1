# round 5: decode kernel -- next tile's DMA spread among the MFMAs (spread), setprio 1 for waves 4-7 (prio), both
set -o pipefail
O=$PWD/gpurun_out/r05v
mkdir -p $O
WAKEWORD_LIB=$PWD/variants/var_sprio/libwakeword.so timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -q -s --timeout 300 --timeout-method thread -k "ctc or config5" > $O/tests.log 2>&1; rc=$?
[ $rc -le 1 ] || { tail -20 $O/tests.log; exit $rc; }
tail -2 $O/tests.log; grep "config5 decisions" $O/tests.log | grep -v print | cut -c1-110
bash tools/debug/ctc_ab.sh spread prio sprio 2>&1 | tee $O/ab.txt
