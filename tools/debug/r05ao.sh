# round 5, K = 32 question: parts of the DFT16 (variant 32 + 256 * part)
# (probe variant 64 + 256 * form; forms in tools/debug/xdl_coresidence_probe.hip)
set -o pipefail
O=$PWD/gpurun_out/r05ao
mkdir -p $O
for v in 1312 2592; do
  timeout -k 10 120 ./tools/debug/xdl_probe 2 20000 $v >> $O/probe12.txt 2>&1 || { cat $O/probe12.txt; exit 1; }
done
grep -v "^workgroup" $O/probe12.txt | cut -c1-160
