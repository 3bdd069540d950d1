# round 5 final check: full GPU suite, headline bench, CTC bench + kernel stats on the final library
set -o pipefail
O=$PWD/gpurun_out/r05w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -20 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json | cut -c1-200
timeout -k 10 300 python bench_ctc.py > $O/ctc.log 2>&1 || exit $?
grep '^{' $O/ctc.log | tail -1 | cut -c1-160
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ctc_trace" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench_ctc.py" --no-cpu-baseline > "$O/ctc_prof.log" 2>&1 || exit $?
