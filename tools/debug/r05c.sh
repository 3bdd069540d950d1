set -o pipefail
O=$PWD/gpurun_out/r05c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -3 $O/gputest.log; grep "config5 decisions\|config5 flipped" $O/gputest.log; timeout -k 10 300 python bench_ctc.py --precision fp16 --steps 5 --no-cpu-baseline > $O/ctc_fp16.json 2> $O/ctc_fp16.err || exit $?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_ctc.py --precision fp32 --steps 5 --no-cpu-baseline > $O/ctc_fp32.json 2> $O/ctc_fp32.err || exit $?
python -c "import json;d=json.loads(open('$O/ctc_fp32.json').read().strip().splitlines()[-1]);print('fp32', d['value'], {k:round(v['ms'],3) for k,v in d['kernels'].items()})"
for v in k16prow k32prow; do
  WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 300 python tools/debug/prow_probe.py bf16 4 >> $O/prow.txt 2>&1 || { cat $O/prow.txt; exit 1; }
done
cat $O/prow.txt
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$i.json 2>&1 || exit $?; tail -1 $O/bench_$i.json | cut -c1-120; done
bash tools/debug/ctc_ab.sh ynt 2>&1 | tee $O/ctc_ynt_ab.txt || exit $?
WAKEWORD_LIB=$PWD/variants/var_ynt/libwakeword.so timeout -k 10 600 bash tools/ctc_pmc.sh r05c_ynt > $O/ctc_pmc_ynt.log 2>&1 || { tail -5 $O/ctc_pmc_ynt.log; exit 1; }
timeout -k 10 600 bash tools/ctc_pmc.sh r05c_prod > $O/ctc_pmc_prod.log 2>&1 || { tail -5 $O/ctc_pmc_prod.log; exit 1; }
grep -h -A3 '"output"' gpurun_out/ctcpmc_r05c_ynt/ctc_hbm_traffic.json gpurun_out/ctcpmc_r05c_prod/ctc_hbm_traffic.json | head -20
