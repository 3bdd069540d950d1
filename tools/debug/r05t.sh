# round 5, K = 32 with SIMD-split roles: bf16 / bf16x3 parity on k32split, bf16x3 repeatability, and speed
set -o pipefail
O=$PWD/gpurun_out/r05t
mkdir -p $O
WAKEWORD_LIB=$PWD/variants/var_k32split/libwakeword.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/k32split_bf16.log 2>&1 || { tail -20 $O/k32split_bf16.log; exit 1; }
tail -2 $O/k32split_bf16.log
WAKEWORD_LIB=$PWD/variants/var_k32split/libwakeword.so timeout -k 10 240 python tools/debug/k32_repeat.py bf16x3 6 > $O/k32split_x3.txt 2>&1 || { cat $O/k32split_x3.txt; exit 1; }
grep -v amdgpu.ids $O/k32split_x3.txt
for v in prod k16split k32split; do
  for p in fp32 bf16 bf16x3; do
    if [ $v = prod ]; then L=$PWD/esp32-wake-word_amd/wakeword/libwakeword.so; else L=$PWD/variants/var_$v/libwakeword.so; fi
    WAKEWORD_LIB=$L timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --precision $p > $O/bench_${v}_$p.json 2>&1 || { tail -5 $O/bench_${v}_$p.json; exit 1; }
    echo "$v $p $(tail -1 $O/bench_${v}_$p.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
