# round 5: output-kernel timing probes (wrong tokens by design): no W DMA after tile 0, minimal epilogue
set -o pipefail
O=$PWD/gpurun_out/r05m
mkdir -p $O
bash tools/debug/ctc_ab.sh nodma noepi 2>&1 | tee $O/ab.txt
