# round 5: the front-end's complex arithmetic as scalar fp32 pairs (-DWK_FE_SCALAR)
# instead of packed v_pk_*_f32: parity of the variant, then A/B fp32 and bf16
set -o pipefail
O=$PWD/gpurun_out/r05au
mkdir -p $O
WAKEWORD_LIB=$PWD/variants/var_fesc/libwakeword.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_bf16.py > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 400 bash tools/debug/ab.sh prod fesc > $O/ab_fp32.txt 2>&1 || { cat $O/ab_fp32.txt; exit 1; }
cat $O/ab_fp32.txt
AB_ARGS="--precision bf16" timeout -k 10 400 bash tools/debug/ab.sh prod fesc > $O/ab_bf16.txt 2>&1 || { cat $O/ab_bf16.txt; exit 1; }
cat $O/ab_bf16.txt
