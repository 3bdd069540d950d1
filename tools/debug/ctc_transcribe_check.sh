#!/bin/bash
# CTC one-call path: GPU tests, then the config-5 bench through wk_ctc_transcribe
# and through the two calls, twice each (through gpurun).
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
O=gpurun_out/tr
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -x -q -k "ctc or config5" \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { tail -30 $O/tests.log; exit $rc; }
for pass in 1 2; do
  for v in one sep; do
    a=""; [ $v = sep ] && a="--separate"
    timeout -k 10 200 python -u bench_ctc.py --no-cpu-baseline $a > $O/ctc_$v.log 2>&1 || { echo "$v failed"; tail -5 $O/ctc_$v.log; exit 1; }
    python -c "import json;d=json.loads(open('$O/ctc_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], 'utt/s', d['ms_per_step'], 'ms', {k: v['ms'] for k, v in d['kernels'].items()})"
  done
done
