# round 5: config 4 (bf16, 131,072 clips per rank) with the scalar-front-end bf16
# unit: bench + rocprofv3 kernel stats; fp32 and bf16x3 benches on the same box
set -o pipefail
O=$PWD/gpurun_out/r05aw
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py --precision bf16 --batch 131072 --no-cpu-baseline > $O/bench_bf16_131k.json 2> $O/b1.err || exit $?
tail -1 $O/bench_bf16_131k.json | cut -c1-120
timeout -k 10 300 python bench.py --precision bf16x3 --no-cpu-baseline > $O/bench_bf16x3.json 2> $O/b2.err || exit $?
tail -1 $O/bench_bf16x3.json | cut -c1-120
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fp32.json 2> $O/b3.err || exit $?
tail -1 $O/bench_fp32.json | cut -c1-120
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --precision bf16 --batch 131072 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/bf16_131k_kernel_stats.csv
head -3 $O/bf16_131k_kernel_stats.csv | cut -c1-150
