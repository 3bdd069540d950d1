set -o pipefail
O=$PWD/gpurun_out/r05b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -3 $O/gputest.log; grep "config5 decisions" $O/gputest.log; [ $rc -eq 0 ] || exit $rc
for p in fp32 fp16; do
  timeout -k 10 300 python bench_ctc.py --precision $p --steps 5 --no-cpu-baseline > $O/ctc_$p.json 2> $O/ctc_$p.err || exit $?
  python -c "import json;d=json.loads(open('$O/ctc_$p.json').read().strip().splitlines()[-1]);print('$p', d['value'], {k:round(v['ms'],3) for k,v in d['kernels'].items()})"
done
WAKEWORD_LIB=$PWD/variants/var_diag/libwakeword.so PRECS="fp32 bf16" bash tools/debug/roles.sh 2>&1 | tee $O/roles.txt || exit $?
WAKEWORD_LIB=$PWD/variants/var_diag/libwakeword.so timeout -k 10 120 python tools/debug/phase_stamps.py 65536 fp32 > $O/stamps_fp32.txt 2>&1 || exit $?
cat $O/stamps_fp32.txt
