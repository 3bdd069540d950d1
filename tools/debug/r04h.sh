set -o pipefail
O=$PWD/gpurun_out/r04h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gputest.log 2>&1; rc=$?; tail -3 $O/gputest.log; [ $rc -eq 0 ] || exit $rc
bash tools/round_bundle.sh r04a || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 180 python bench.py --no-cpu-baseline --precision bf16 --batch 131072 > $O/bench_bf16_131k.log 2>&1 || exit $?
tail -1 $O/bench_bf16_131k.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --precision bf16 --batch 131072 > $O/c4_prof.log 2>&1 || exit $?
echo c4 profiled
