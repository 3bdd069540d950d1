set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gruabl && cd /tmp && export TMPDIR=/tmp
for v in prod abl1 abl2 abl3; do
  if [ $v = prod ]; then L=$GRAFT_REPO_ROOT/esp32-wake-word_amd/wakeword/libwakeword.so; else L=$GRAFT_REPO_ROOT/esp32-wake-word_amd/build/var_$v/libwakeword.so; fi
  WAKEWORD_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gruabl/$v -o run -- python3 $GRAFT_REPO_ROOT/bench_ctc.py --steps 3 --cpu-utts 1 > $GRAFT_REPO_ROOT/gpurun_out/gruabl/$v.log 2>&1 || exit 1
done
