set -o pipefail
O=$PWD/gpurun_out/r04l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -3 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench_ctc.py > $O/ctc.log 2>&1 || exit $?
grep '^{' $O/ctc.log | tail -1 | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ctc_trace -o run -- python3 $GRAFT_REPO_ROOT/bench_ctc.py --no-cpu-baseline > $O/ctc_prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python bench.py > $O/bench_fp32.log 2>&1 || exit $?
tail -1 $O/bench_fp32.log | cut -c1-200
timeout -k 10 600 bash tools/ctc_pmc.sh r04b > $O/ctc_pmc.log 2>&1 || { echo "ctc pmc failed"; tail -5 $O/ctc_pmc.log; exit 1; }
tail -20 $O/ctc_pmc.log
bash tools/debug/ab.sh prod dppord 2>&1 | tee $O/ab.txt
