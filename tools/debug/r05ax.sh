# round 5: rocprofv3 kernel stats of config 4 (bf16, 131,072 clips) with the
# scalar-front-end bf16 unit (r05aw had the output format wrong)
set -o pipefail
O=$PWD/gpurun_out/r05ax
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --precision bf16 --batch 131072 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/bf16_131k_kernel_stats.csv
head -3 $O/bf16_131k_kernel_stats.csv | cut -c1-150
tail -1 $O/prof.log | cut -c1-120
