# round 5, K = 32 question: the standalone probe with the front-end's DFT16 as
# the VALU work (variant bit 32; +16 sparse MFMA stream, +4 MFMA-side LDS traffic)
set -o pipefail
O=$PWD/gpurun_out/r05an
mkdir -p $O
for v in 32 48 36; do
  timeout -k 10 120 ./tools/debug/xdl_probe 2 20000 $v >> $O/probe5.txt 2>&1 || { cat $O/probe5.txt; exit 1; }
done
grep -v "^workgroup" $O/probe5.txt
