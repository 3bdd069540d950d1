# round 5: encoder prefetch depth 2 / 3 (pf2, pf3) A/B against the product
set -o pipefail
O=$PWD/gpurun_out/r05i
mkdir -p $O
bash tools/debug/ctc_ab.sh pf2 pf3 2>&1 | tee $O/ab.txt
