# round 5: config-5 repeatability at scale (the new test) + the existing repeat tests
set -o pipefail
O=$PWD/gpurun_out/r05ah
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider \
  tests/test_gpu_configs.py::test_config5_repeatable_at_scale tests/test_ctc.py::test_ctc_bit_repeatable_at_scale \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
