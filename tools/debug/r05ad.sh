# round 5: decode kernel fragment prefetch distance 6 / 3 and the fold spread over 3 of every 4 steps
set -o pipefail
O=$PWD/gpurun_out/r05ad
mkdir -p $O
bash tools/debug/ctc_ab.sh pd6 spread pd3 2>&1 | tee $O/ab.txt
