set -o pipefail
O=gpurun_out/extra_r03f
mkdir -p $O
timeout -k 10 300 python bench_stream.py > $O/stream.log 2>&1 || exit $?
timeout -k 10 300 python bench_surfaces.py > $O/surfaces.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16x3 > $O/bench_bf16x3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --audio i16 --precision bf16 > $O/bench_bf16_i16.log 2>&1 || exit $?
for f in stream surfaces bench_bf16x3 bench_bf16_i16; do echo "$f: $(grep '^{' $O/$f.log | tail -1 | cut -c1-400)"; done
