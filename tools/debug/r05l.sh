# round 5 final bundle, part 2: streaming / CTC / surfaces / bf16x3 benches + CTC kernel stats, then CTC PMC
set -o pipefail
R=$PWD
O=$R/gpurun_out/extra_r05
mkdir -p "$O"
timeout -k 10 300 python bench_stream.py > "$O/stream.log" 2>&1 || exit $?
timeout -k 10 300 python bench_ctc.py > "$O/ctc.log" 2>&1 || exit $?
timeout -k 10 300 python bench_ctc.py --precision fp32 > "$O/ctc_fp32.log" 2>&1 || exit $?
timeout -k 10 300 python bench_surfaces.py > "$O/surfaces.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16x3 > "$O/bench_bf16x3.log" 2>&1 || exit $?
for f in stream ctc ctc_fp32 surfaces bench_bf16x3; do echo "$f: $(grep '^{' $O/$f.log | tail -1 | cut -c1-200)"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ctc_trace" -o run -- \
  python3 "$R/bench_ctc.py" --no-cpu-baseline > "$O/ctc_prof.log" 2>&1 || exit $?
cd "$R"
timeout -k 10 900 bash tools/ctc_pmc.sh r05 > gpurun_out/ctcpmc_r05.log 2>&1 || { tail -5 gpurun_out/ctcpmc_r05.log; exit 1; }
tail -3 gpurun_out/ctcpmc_r05.log
