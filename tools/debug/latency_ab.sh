#!/bin/bash
# Single-window latency A/B (stream_lat.py) and throughput A/B of the in-tree library against variants/var_head, after the GPU tests that exercise short batches.
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_stream.py tests/test_gpu_bf16.py tests/test_gpu_configs.py tests/test_gpu_protocol.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do for v in prod head; do
  if [ $v = prod ]; then L=esp32-wake-word_amd/wakeword/libwakeword.so; else L=variants/var_head/libwakeword.so; fi
  WAKEWORD_LIB=$L timeout -k 10 120 python tools/debug/stream_lat.py > $O/lat_${v}_$pass.txt 2>&1 || exit $?
  echo "$v pass $pass: $(grep -E 'batch 1|C call' $O/lat_${v}_$pass.txt | tr '\n' ' ')"
done; done
bash tools/debug/ab.sh prod head > $O/ab.txt 2>&1 || exit $?
AB_ARGS="--precision bf16" bash tools/debug/ab.sh prod head >> $O/ab.txt 2>&1 || exit $?
cat $O/ab.txt
