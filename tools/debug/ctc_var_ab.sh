#!/bin/bash
# CTC A/B with per-variant parity: for each build/var_<name> (and "prod"), the
# fp16 fused-projection CTC tests through that library, then the config-5
# bench, twice round-robin.
#   bash tools/debug/ctc_var_ab.sh <variant...>   (through gpurun)
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
mkdir -p gpurun_out/ab
# a variant named env_NAME=VAL runs the in-tree library with that environment variable set
libof() { case "$1" in prod|env_*) echo "$R/esp32-wake-word_amd/wakeword/libwakeword.so";; *) echo "$R/variants/var_$1/libwakeword.so";; esac; }
envof() { case "$1" in env_*) echo "${1#env_}";; *) echo "WK_AB_NONE=1";; esac; }
for v in prod "$@"; do
  case "$v" in abl_*) echo "$v: ablation (wrong results by design), tests skipped"; continue;; esac
  K="fp16 or config5"; [ $v = prod ] && K="ctc or config"   # the in-tree library gets every CTC test
  env $(envof $v) WAKEWORD_LIB=$(libof $v) timeout -k 10 200 python -u -m pytest tests/test_ctc.py tests/test_gpu_configs.py -m gpu -x -q \
    -k "$K" --timeout 120 --timeout-method thread > gpurun_out/ab/tests_$v.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/ab/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for pass in 1 2; do
  for v in prod "$@"; do
    env $(envof $v) WAKEWORD_LIB=$(libof $v) timeout -k 10 200 python -u bench_ctc.py --no-cpu-baseline $CTC_ARGS > gpurun_out/ab/ctc_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab/ctc_$v.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab/ctc_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], 'utt/s', d['ms_per_step'], 'ms', {k: v['ms'] for k, v in d['kernels'].items()})"
  done
done
