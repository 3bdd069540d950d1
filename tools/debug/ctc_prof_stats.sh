set -o pipefail
mkdir -p gpurun_out/ctcprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ctcprof/trace -o run -- python3 $GRAFT_REPO_ROOT/bench_ctc.py --steps 5 --cpu-utts 1 > $GRAFT_REPO_ROOT/gpurun_out/ctcprof/bench.log 2>&1
