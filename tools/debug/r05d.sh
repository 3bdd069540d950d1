set -o pipefail
O=$PWD/gpurun_out/r05d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -v -s -x --timeout 300 --timeout-method thread > $O/ctctest.log 2>&1; rc=$?; tail -3 $O/ctctest.log; grep "config5" $O/ctctest.log; [ $rc -eq 0 ] || exit $rc
for p in fp32 fp16; do
  timeout -k 10 300 python bench_ctc.py --precision $p --steps 5 --no-cpu-baseline > $O/ctc_$p.json 2> $O/ctc_$p.err || exit $?
  python -c "import json;d=json.loads(open('$O/ctc_$p.json').read().strip().splitlines()[-1]);print('$p', d['value'], {k:round(v['ms'],3) for k,v in d['kernels'].items()})"
done
for v in k16prow k32prow; do
  WAKEWORD_LIB=$PWD/variants/var_$v/libwakeword.so timeout -k 10 400 python tools/debug/prow_probe.py bf16 4 >> $O/prow.txt 2>&1 || { cat $O/prow.txt; exit 1; }
done
grep -v amdgpu.ids $O/prow.txt
