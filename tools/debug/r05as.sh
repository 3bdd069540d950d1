# round 5: int8 matrix-core kernel at scale (the new repeatability test) + its file
set -o pipefail
O=$PWD/gpurun_out/r05as
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_int8.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/tests.log
