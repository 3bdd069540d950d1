# round 5: product library with the decode-only output kernel: full GPU suite + CTC bench + kernel stats
set -o pipefail
O=$PWD/gpurun_out/r05q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -20 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log; grep "config5 decisions" $O/gputest.log | grep -v print
timeout -k 10 300 python bench_ctc.py > $O/ctc.log 2>&1 || exit $?
grep '^{' $O/ctc.log | tail -1 | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ctc_trace" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench_ctc.py" --no-cpu-baseline > "$O/ctc_prof.log" 2>&1 || exit $?
