set -o pipefail
O=$PWD/gpurun_out/r04j
mkdir -p $O
bash tools/debug/ab.sh prod sl1 sl4 sl8 poll poll4 2>&1 | tee $O/ab.txt
