#!/bin/bash
# CTC A/B (config 5 bench, fp16) of the in-tree library ("prod") against
# build/var_<name> variants, after the CTC tests on the in-tree library.
#   bash tools/debug/ctc_ab.sh <variant...>
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ctc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ctc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ctc_tests.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for v in prod "$@"; do
    if [ "$v" = prod ]; then L=$R/esp32-wake-word_amd/wakeword/libwakeword.so; else L=$R/variants/var_$v/libwakeword.so; fi
    WAKEWORD_LIB=$L timeout -k 10 200 python -u bench_ctc.py --cpu-utts 1 $CTC_ARGS > gpurun_out/ctc_ab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ctc_ab_$v.log; exit 1; }
    python - "$v" gpurun_out/ctc_ab_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], "utt/s", d["ms_per_step"], "ms", {k: v["ms"] for k, v in d["kernels"].items()})
PY
  done
done
