set -o pipefail
O=$PWD/gpurun_out/r05a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -3 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/debug/ab.sh prod base prod base 2>&1 | tee $O/ab.txt || exit $?
for v in k32 k32pad; do
  WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 240 python tools/debug/k32_repeat.py bf16 6 feats >> $O/k32.txt 2>&1 || exit $?
done
cat $O/k32.txt
bash tools/pmc_census.sh $O/census_prod > $O/census_prod.log 2>&1 || exit $?
WAKEWORD_LIB=$PWD/variants/var_base/libwakeword.so bash tools/pmc_census.sh $O/census_base > $O/census_base.log 2>&1 || exit $?
python tools/pmc_census.py $O/census_prod > $O/census_prod.txt 2>&1
python tools/pmc_census.py $O/census_base > $O/census_base.txt 2>&1
grep -h "SQ_INSTS \|SQ_INSTS_MFMA\|MFMA_BUSY\|SQ_INSTS_VALU \|kernel_cycles" $O/census_prod.txt $O/census_base.txt
for v in prod base; do
  L=$PWD/esp32-wake-word_amd/wakeword/libwakeword.so; [ $v = base ] && L=$PWD/variants/var_base/libwakeword.so
  WAKEWORD_LIB=$L timeout -k 10 300 python bench_ctc.py --precision fp32 --steps 3 --no-cpu-baseline > $O/ctc_fp32_$v.json 2> $O/ctc_fp32_$v.err || exit $?
  tail -1 $O/ctc_fp32_$v.json | cut -c1-300
done
