set -o pipefail
O=$PWD/gpurun_out/r04u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -2 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 240 python bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-160
