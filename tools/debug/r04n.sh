set -o pipefail
O=$PWD/gpurun_out/r04n
mkdir -p $O
bash tools/debug/ctc_ab.sh outnt 2>&1 | tee $O/ctc_ab.txt || exit 1
cd /tmp && export TMPDIR=/tmp
for v in prod outnt; do
  if [ $v = prod ]; then L=$GRAFT_REPO_ROOT/esp32-wake-word_amd/wakeword/libwakeword.so; else L=$GRAFT_REPO_ROOT/variants/var_$v/libwakeword.so; fi
  WAKEWORD_LIB=$L timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_$v -o run -- python3 $GRAFT_REPO_ROOT/bench_ctc.py --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_$v.log 2>&1 || exit 1
done
