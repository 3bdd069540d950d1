# round 5, K = 32 question: the minimal co-residence probe (no fused kernel),
# VALU/MFMA instruction-mix variants (tools/debug/xdl_coresidence_probe.hip);
# xdl_probe28: 28 packed chains per lane, 122 VGPRs (the front-end's register range)
set -o pipefail
O=$PWD/gpurun_out/r05ai
mkdir -p $O
for v in 0 15 31; do
  timeout -k 10 120 ./tools/debug/xdl_probe28 2 10000 $v >> $O/probe4.txt 2>&1 || { cat $O/probe4.txt; exit 1; }
done
grep -v "^workgroup" $O/probe4.txt
