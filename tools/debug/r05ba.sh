# round 5 final: the product with the bf16 family on K = 32 beside its scalar-fp32
# front-end: GPU suite, K = 32 repeatability at scale, benches (fp32, bf16 at
# config 4's 131,072 clips, bf16x3), CTC bench
set -o pipefail
O=$PWD/gpurun_out/r05ba
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputest.log 2>&1 || { tail -20 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for p in bf16 bf16x3; do
  timeout -k 10 240 python tools/debug/k32_repeat.py $p 6 feats >> $O/k32.txt 2>&1 || { cat $O/k32.txt; exit 1; }
done
grep -v amdgpu.ids $O/k32.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/b0.err || exit $?
tail -1 $O/bench.json | cut -c1-130
timeout -k 10 300 python bench.py --precision bf16 --batch 131072 --no-cpu-baseline > $O/bench_bf16_131k.json 2> $O/b1.err || exit $?
tail -1 $O/bench_bf16_131k.json | cut -c1-130
timeout -k 10 300 python bench.py --precision bf16x3 --no-cpu-baseline > $O/bench_bf16x3.json 2> $O/b2.err || exit $?
tail -1 $O/bench_bf16x3.json | cut -c1-130
timeout -k 10 300 python bench_ctc.py > $O/ctc.log 2>&1 || exit $?
grep '^{' $O/ctc.log | tail -1 | cut -c1-130
