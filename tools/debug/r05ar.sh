# round 5, K = 32 question: the product's other MFMA forms beside the reproducing
# VALU loops -- fp32 v_mfma_f32_16x16x4_f32 (mode 7), int8 v_mfma_i32_16x16x64_i8 (mode 8)
set -o pipefail
O=$PWD/gpurun_out/r05ar
mkdir -p $O
for v in 1312 32; do
  XDL_PROBE_MODES=01278 timeout -k 10 120 ./tools/debug/xdl_probe 2 20000 $v >> $O/probe14.txt 2>&1 || { cat $O/probe14.txt; exit 1; }
done
grep -v "^workgroup" $O/probe14.txt | sed 's/by lane:.*by output float/by output float/' | cut -c1-200
