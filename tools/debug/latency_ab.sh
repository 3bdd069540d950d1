#!/bin/bash
# Single-window latency A/B (stream_lat.py, bench_stream.py) of the in-tree library against
# variants/var_head, after the GPU tests that exercise short batches and the stream.
#   OUT=gpurun_out/<dir> [THROUGHPUT=1] bash tools/debug/latency_ab.sh
set -o pipefail
O=${OUT:-gpurun_out/lat_ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_stream.py tests/test_gpu_bf16.py tests/test_gpu_configs.py tests/test_gpu_protocol.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do for v in prod head; do
  if [ $v = prod ]; then L=esp32-wake-word_amd/wakeword/libwakeword.so; else L=variants/var_head/libwakeword.so; fi
  WAKEWORD_LIB=$L timeout -k 10 120 python tools/debug/stream_lat.py > $O/lat_${v}_$pass.txt 2>&1 || exit $?
  WAKEWORD_LIB=$L timeout -k 10 300 python bench_stream.py > $O/stream_${v}_$pass.json 2>&1 || exit $?
  echo "$v pass $pass: $(grep -E 'batch 1|C call|Detector' $O/lat_${v}_$pass.txt | tr '\n' ' ')"
  echo "   bench_stream: $(tail -1 $O/stream_${v}_$pass.json)"
done; done
[ -n "$THROUGHPUT" ] || exit 0
bash tools/debug/ab.sh prod head > $O/ab.txt 2>&1 || exit $?
AB_ARGS="--precision bf16" bash tools/debug/ab.sh prod head >> $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
