set -o pipefail
mkdir -p gpurun_out/r03g
timeout -k 10 300 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03g/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03g/tests.log
timeout -k 10 200 python bench_ctc.py --no-cpu-baseline > gpurun_out/r03g/ctc_fused.log 2>&1 || exit $?
WAKEWORD_CTC_GEMM=1 timeout -k 10 200 python bench_ctc.py --no-cpu-baseline > gpurun_out/r03g/ctc_gemm.log 2>&1 || exit $?
for f in fused gemm; do python -c "
import json; d=json.loads(open('gpurun_out/r03g/ctc_$f.log').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()})"; done
exit $rc
