# round 5 probe: the decode kernel's per-period barrier (nobar: timing only, wrong tokens) -- kernel stats vs prod
set -o pipefail
O=$PWD/gpurun_out/r05x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in prod nobar; do
  if [ $v = prod ]; then L=$GRAFT_REPO_ROOT/esp32-wake-word_amd/wakeword/libwakeword.so; else L=$GRAFT_REPO_ROOT/variants/var_$v/libwakeword.so; fi
  WAKEWORD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$v" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench_ctc.py" --no-cpu-baseline > "$O/$v.log" 2>&1 || exit $?
  grep decode16 $O/$v/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-60,140-220
done
