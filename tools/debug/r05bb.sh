# round 5: the fp32 unit with only the DFT16s in scalar fp32 (-DWK_FE_DFT_SCALAR),
# the rest of the front-end packed: parity, then A/B fp32 (three passes)
set -o pipefail
O=$PWD/gpurun_out/r05bb
mkdir -p $O
WAKEWORD_LIB=$PWD/variants/var_ds/libwakeword.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_parity.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 400 bash tools/debug/ab.sh prod ds > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
timeout -k 10 400 bash tools/debug/ab.sh prod ds >> $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
