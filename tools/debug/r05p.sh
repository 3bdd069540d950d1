# round 5: decode-kernel variants (prefetch distance 4, free scheduling) A/B against prod and dec16b
set -o pipefail
O=$PWD/gpurun_out/r05p
mkdir -p $O
bash tools/debug/ctc_ab.sh dec16b dec16c dec16d dec16e dec16f 2>&1 | tee $O/ab.txt
