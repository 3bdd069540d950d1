# round 5: K = 32 bf16 MFMA in the bf16-family fused unit (scalar-fp32 front-end),
# -DWK_XDL_K32: parity + bf16 suites, features repeatability, A/B against the product
set -o pipefail
O=$PWD/gpurun_out/r05az
mkdir -p $O
L=$PWD/variants/var_x32/libwakeword.so
WAKEWORD_LIB=$L timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_configs.py::test_config4_bf16_rank_shard > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for p in bf16 bf16x3; do
  WAKEWORD_LIB=$L timeout -k 10 240 python tools/debug/k32_repeat.py $p 6 feats >> $O/k32.txt 2>&1 || { cat $O/k32.txt; exit 1; }
done
grep -v amdgpu.ids $O/k32.txt
for p in bf16 bf16x3; do
  echo "== $p" >> $O/ab.txt
  AB_ARGS="--precision $p" timeout -k 10 400 bash tools/debug/ab.sh prod x32 >> $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
done
cat $O/ab.txt
