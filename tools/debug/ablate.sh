# WAKEWORD_FUSED_EXP needs variants built with -DWK_DEBUG_EXPERIMENTS (the shipped library ignores it).
cd $GRAFT_REPO_ROOT
for v in prod ${ABL_VARIANTS:-abl_NODFT abl_NOTW abl_NOTRANS abl_NOSPLIT abl_NOMEL}; do
  if [ $v = prod ]; then L=esp32-wake-word_amd/wakeword/libwakeword.so; else L=esp32-wake-word_amd/build/var_$v/libwakeword.so; fi
  WAKEWORD_LIB=$L WAKEWORD_FUSED_EXP=1 timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --precision bf16 > gpurun_out/abl_$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/abl_$v.log').read().strip().splitlines()[-1]);print('$v', d['roofline']['launch_ms'])"
done
