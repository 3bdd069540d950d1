export WAKEWORD_LIB=$PWD/esp32-wake-word_amd/build/var_exp/libwakeword.so
for cfg in "fp32 0" "fp32 1" "fp32 2" "bf16 0"; do
  set -- $cfg
  WAKEWORD_FUSED_EXP=$2 bash tools/debug/pmc_groups.sh gpurun_out/pmc_$1_$2 tools/debug/groups_issue.txt --steps 2 --warmup 1 --no-cpu-baseline --precision $1 || exit 1
done
