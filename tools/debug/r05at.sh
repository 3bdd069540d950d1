# round 5 final tree (int8 at-scale test added): GPU suite + headline bench + CTC bench
set -o pipefail
O=$PWD/gpurun_out/r05at
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -20 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json | cut -c1-150
timeout -k 10 300 python bench_ctc.py > $O/ctc.log 2>&1 || exit $?
grep '^{' $O/ctc.log | tail -1 | cut -c1-150
