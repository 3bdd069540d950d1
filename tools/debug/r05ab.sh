# round 5 final CTC bundle on the final library: GPU suite, bench_ctc (fp16, fp32) + kernel stats, CTC PMC
set -o pipefail
O=$PWD/gpurun_out/r05ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -20 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python bench_ctc.py > $O/ctc.log 2>&1 || exit $?
timeout -k 10 300 python bench_ctc.py --precision fp32 > $O/ctc_fp32.log 2>&1 || exit $?
grep '^{' $O/ctc.log | tail -1 | cut -c1-160
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench_ctc.py" --no-cpu-baseline > "$O/prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 bash tools/ctc_pmc.sh r05ab > gpurun_out/ctcpmc_r05ab.log 2>&1 || { tail -5 gpurun_out/ctcpmc_r05ab.log; exit 1; }
tail -12 gpurun_out/ctcpmc_r05ab.log
